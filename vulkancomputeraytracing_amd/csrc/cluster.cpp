// cluster.cpp -- k-d grouping of spheres into fours + conservative group bounds (cluster.hpp).
#include "cluster.hpp"

#include <algorithm>
#include <array>
#include <cmath>
#include <limits>

namespace vcrt {
namespace {

// Smallest float >= x (x finite, double).
float round_up(double x) {
    float f = static_cast<float>(x);
    if (static_cast<double>(f) < x) f = std::nextafter(f, std::numeric_limits<float>::infinity());
    return f;
}

using Group = std::array<int32_t, 4>;

// Median splits on the widest centre axis; the left part always holds a multiple of four
// spheres so only the last leaf of a run is padded.
void split(std::vector<int32_t>& idx, size_t lo, size_t hi, const vcrt_sphere* s,
           std::vector<Group>& groups) {
    const size_t n = hi - lo;
    if (n <= 4) {
        Group g{-1, -1, -1, -1};
        for (size_t k = 0; k < n; k++) g[k] = idx[lo + k];
        groups.push_back(g);
        return;
    }
    double mn[3], mx[3];
    for (int a = 0; a < 3; a++) {
        mn[a] = std::numeric_limits<double>::infinity();
        mx[a] = -mn[a];
    }
    for (size_t k = lo; k < hi; k++)
        for (int a = 0; a < 3; a++) {
            mn[a] = std::min(mn[a], static_cast<double>(s[idx[k]].center[a]));
            mx[a] = std::max(mx[a], static_cast<double>(s[idx[k]].center[a]));
        }
    int axis = 0;
    for (int a = 1; a < 3; a++)
        if (mx[a] - mn[a] > mx[axis] - mn[axis]) axis = a;
    const size_t ng = (n + 3) / 4;
    const size_t mid = lo + 4 * ((ng + 1) / 2);
    std::nth_element(idx.begin() + lo, idx.begin() + mid, idx.begin() + hi,
                     [&](int32_t x, int32_t y) {
                         const float cx = s[x].center[axis], cy = s[y].center[axis];
                         return cx < cy || (cx == cy && x < y);
                     });
    split(idx, lo, mid, s, groups);
    split(idx, mid, hi, s, groups);
}

}  // namespace

bool build_cull_tables(const vcrt_sphere* s, int32_t count, CullTables& out) {
    out = CullTables{};
    if (count < 16) return false;
    for (int32_t i = 0; i < count; i++)
        for (float v : {s[i].center[0], s[i].center[1], s[i].center[2], s[i].radius})
            if (!(std::fabs(v) <= 0x1p30f)) return false;

    // Very large spheres (the ground) would inflate any group they join: group them apart.
    std::vector<float> radii(count);
    for (int32_t i = 0; i < count; i++) radii[i] = std::fabs(s[i].radius);
    std::vector<float> sorted = radii;
    std::nth_element(sorted.begin(), sorted.begin() + count / 2, sorted.end());
    const float huge = 8.0f * sorted[count / 2];
    std::vector<int32_t> normal, big;
    for (int32_t i = 0; i < count; i++) (radii[i] > huge ? big : normal).push_back(i);
    std::vector<Group> groups;
    if (!normal.empty()) split(normal, 0, normal.size(), s, groups);
    if (!big.empty()) split(big, 0, big.size(), s, groups);
    if (groups.size() % 2) groups.push_back(Group{-1, -1, -1, -1});

    const size_t ng = groups.size();
    out.ngroups = static_cast<int32_t>(ng);
    out.geom.assign(ng * 16, 0.0f);
    out.bound.assign(ng / 2 * 16, 0.0f);
    out.index.assign(ng * 4, -1);
    for (size_t gi = 0; gi < ng; gi++) {
        const Group& g = groups[gi];
        // members: pair-SoA exactly as the linear table (r^2 = radius * radius in fp32)
        for (int k = 0; k < 4; k++) {
            float* base = &out.geom[gi * 16 + 8 * (k / 2)];
            const int e = k % 2;
            float cx = 0.f, cy = 0.f, cz = 0.f, r2 = -3.0e38f;
            if (g[k] >= 0) {
                const vcrt_sphere& sp = s[g[k]];
                cx = sp.center[0];
                cy = sp.center[1];
                cz = sp.center[2];
                r2 = sp.radius * sp.radius;
            }
            base[0 + e] = cx;
            base[2 + e] = cy;
            base[4 + e] = cz;
            base[6 + e] = r2;
            out.index[gi * 4 + k] = g[k];
        }
        // bound: centre of the members' box (rounded to fp32 first), radius covering every
        // member from that fp32 centre, margin coefficient Kc = 2*8*17u / r_min (tracer.hip)
        float C[3] = {0.f, 0.f, 0.f}, R = 0.f, Rsq = 0.f, Kc = 0.f;
        if (g[0] >= 0) {
            double lo[3], hi[3];
            for (int a = 0; a < 3; a++) {
                lo[a] = std::numeric_limits<double>::infinity();
                hi[a] = -lo[a];
            }
            double rmin = std::numeric_limits<double>::infinity();
            for (int k = 0; k < 4 && g[k] >= 0; k++) {
                const vcrt_sphere& sp = s[g[k]];
                const double r = std::fabs(static_cast<double>(sp.radius));
                rmin = std::min(rmin, r);
                for (int a = 0; a < 3; a++) {
                    lo[a] = std::min(lo[a], sp.center[a] - r);
                    hi[a] = std::max(hi[a], sp.center[a] + r);
                }
            }
            for (int a = 0; a < 3; a++) C[a] = static_cast<float>(0.5 * (lo[a] + hi[a]));
            double rad = 0.0;
            for (int k = 0; k < 4 && g[k] >= 0; k++) {
                const vcrt_sphere& sp = s[g[k]];
                double d2 = 0.0;
                for (int a = 0; a < 3; a++) {
                    const double d = static_cast<double>(sp.center[a]) - C[a];
                    d2 += d * d;
                }
                rad = std::max(rad, std::sqrt(d2) + std::fabs(static_cast<double>(sp.radius)));
            }
            rad *= 1.0 + 1e-6;
            R = round_up(rad);
            Rsq = round_up(static_cast<double>(R) * R);
            Kc = rmin >= 1e-3 ? round_up(1.62e-5 / rmin) : std::numeric_limits<float>::infinity();
        }
        float* b = &out.bound[(gi / 2) * 16];
        const int e = gi % 2;
        b[0 + e] = C[0];
        b[2 + e] = C[1];
        b[4 + e] = C[2];
        b[6 + e] = R;
        b[8 + e] = Rsq;
        b[10 + e] = Kc;
    }
    return true;
}

}  // namespace vcrt
