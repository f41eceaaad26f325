// cluster.cpp -- k-d grouping of spheres into fours + conservative group boxes (cluster.hpp).
#include "cluster.hpp"

#include <algorithm>
#include <array>
#include <cmath>
#include <cstdlib>
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

// Median splits on the widest centre axis. The left part gets ceil(groups / 2) groups rounded
// up to a multiple of 64 (more than 64 groups) or 8 (more than 8), so every subtree starts on a
// node (8 groups) and chunk (64 groups) boundary and nodes are whole subtrees; only the last
// leaf is partial.
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
    const size_t align = ng > 64 ? 64 : ng > 8 ? 8 : 1;
    const size_t left = ((ng + 1) / 2 + align - 1) / align * align;
    const size_t mid = lo + 4 * left;
    std::nth_element(idx.begin() + lo, idx.begin() + mid, idx.begin() + hi,
                     [&](int32_t x, int32_t y) {
                         const float cx = s[x].center[axis], cy = s[y].center[axis];
                         return cx < cy || (cx == cy && x < y);
                     });
    split(idx, lo, mid, s, groups);
    split(idx, mid, hi, s, groups);
}

constexpr double kU = 0x1p-24;  // fp32 unit roundoff

// Smallest float <= x (x finite, double).
float round_down(double x) {
    float f = static_cast<float>(x);
    if (static_cast<double>(f) > x) f = std::nextafter(f, -std::numeric_limits<float>::infinity());
    return f;
}

struct Box {
    float lo[3] = {1e20f, 1e20f, 1e20f};  // padding: a point far away (its groups are empty)
    float hi[3] = {1e20f, 1e20f, 1e20f};
    float K = 0.0f;                       // margin factor 8.1u / r_min of the members
};

// Axis-aligned box of `members` (centre -+ |radius|, rounded outwards to fp32) and its margin
// factor K = 8.1u / r_min (1 + 1e-5), rounded up (inf for a zero radius: never ruled out).
Box box_of(const vcrt_sphere* s, const std::vector<int32_t>& members) {
    Box b;
    if (members.empty()) return b;
    double rmin = std::numeric_limits<double>::infinity();
    for (int32_t j : members) rmin = std::min(rmin, std::fabs(static_cast<double>(s[j].radius)));
    b.K = rmin > 0.0 ? round_up(std::min(8.1 * kU / rmin * (1.0 + 1e-5), 1e38))
                     : std::numeric_limits<float>::infinity();
    for (int a = 0; a < 3; a++) {
        double lo = std::numeric_limits<double>::infinity(), hi = -lo;
        for (int32_t j : members) {
            const double r = std::fabs(static_cast<double>(s[j].radius));
            lo = std::min(lo, s[j].center[a] - r);
            hi = std::max(hi, s[j].center[a] + r);
        }
        b.lo[a] = round_down(lo);
        b.hi[a] = round_up(hi);
    }
    return b;
}

// Element i of a pair-SoA box table (TraceParams.cbound / cnode / ctop):
//   (lox0,lox1,loy0,loy1) (loz0,loz1,hix0,hix1) (hiy0,hiy1,hiz0,hiz1) (K0,K1,0,0)
void put_box(std::vector<float>& table, size_t i, const Box& b) {
    float* t = &table[(i / 2) * 16];
    const int e = i % 2;
    t[0 + e] = b.lo[0];
    t[2 + e] = b.lo[1];
    t[4 + e] = b.lo[2];
    t[6 + e] = b.hi[0];
    t[8 + e] = b.hi[1];
    t[10 + e] = b.hi[2];
    t[12 + e] = b.K;
}

}  // namespace

bool build_cull_tables(const vcrt_sphere* s, int32_t count, CullTables& out) {
    out = CullTables{};
    if (count < 16) return false;
    for (int32_t i = 0; i < count; i++)
        for (float v : {s[i].center[0], s[i].center[1], s[i].center[2], s[i].radius})
            if (!(std::fabs(v) <= 0x1p30f)) return false;

    // Very large spheres (the ground) would inflate any group they join: a sphere is big when
    // its radius exceeds both 8x the median and 5% of the extent of all centres; at most the
    // 64 largest go to the big list (tested for every ray), the rest stay in the hierarchy.
    std::vector<float> radii(count);
    for (int32_t i = 0; i < count; i++) radii[i] = std::fabs(s[i].radius);
    std::vector<float> sorted = radii;
    std::nth_element(sorted.begin(), sorted.begin() + count / 2, sorted.end());
    double lo[3], hi[3];
    for (int a = 0; a < 3; a++) {
        lo[a] = std::numeric_limits<double>::infinity();
        hi[a] = -lo[a];
    }
    for (int32_t i = 0; i < count; i++)
        for (int a = 0; a < 3; a++) {
            lo[a] = std::min(lo[a], static_cast<double>(s[i].center[a]));
            hi[a] = std::max(hi[a], static_cast<double>(s[i].center[a]));
        }
    const double extent = std::sqrt((hi[0] - lo[0]) * (hi[0] - lo[0]) +
                                    (hi[1] - lo[1]) * (hi[1] - lo[1]) +
                                    (hi[2] - lo[2]) * (hi[2] - lo[2]));
    const double huge = std::max(8.0 * sorted[count / 2], 0.05 * extent);
    std::vector<int32_t> normal, big;
    for (int32_t i = 0; i < count; i++) (radii[i] > huge ? big : normal).push_back(i);
    if (big.size() > 64) {  // keep the 64 largest (ties by index), return the rest
        std::stable_sort(big.begin(), big.end(),
                         [&](int32_t x, int32_t y) { return radii[x] > radii[y]; });
        normal.insert(normal.end(), big.begin() + 64, big.end());
        big.resize(64);
        std::sort(big.begin(), big.end());
    }
    // The big list's last group has free slots when the big spheres are not a multiple of four;
    // the largest of the rest fill them (ties by index). Every ray tests that group's members
    // anyway, while in the hierarchy a large sphere inflates the boxes of its group, node and
    // chunk for every ray that passes near it: the final scene's big three (radius 1, beside 480
    // of radius 0.2) join the ground, C4 +9% (same bits). It also keeps the stress scene's
    // hierarchy (4096 random spheres) within the flat scans' 1024 16-bit groups.
    // VCRT_BIG_FILL=0 disables it (A/B).
    const size_t free_slots = (4 - big.size() % 4) % 4;
    const char* fill_env = std::getenv("VCRT_BIG_FILL");
    const bool fill = !(fill_env && std::atoi(fill_env) == 0);
    if (fill && !big.empty() && free_slots > 0 && normal.size() > free_slots) {
        std::stable_sort(normal.begin(), normal.end(),
                         [&](int32_t x, int32_t y) { return radii[x] > radii[y]; });
        big.insert(big.end(), normal.begin(), normal.begin() + free_slots);
        normal.erase(normal.begin(), normal.begin() + free_slots);
        std::sort(big.begin(), big.end());
        std::sort(normal.begin(), normal.end());
    }
    // Big spheres go to a short list the kernels test for every ray (they are hit by most);
    // the rest form the hierarchy: groups of 4, nodes of 8 groups, chunks of 64 groups.
    std::vector<Group> bigg, groups;
    if (!big.empty()) split(big, 0, big.size(), s, bigg);
    if (!normal.empty()) split(normal, 0, normal.size(), s, groups);
    // pad the hierarchy to whole nodes and an even node count (pair layout)
    while (groups.size() % (2 * kNodeGroups)) groups.push_back(Group{-1, -1, -1, -1});

    const size_t nbig = bigg.size(), ng = groups.size(), nall = nbig + ng;
    out.nbig = static_cast<int32_t>(nbig);
    out.ngroups = static_cast<int32_t>(ng);
    out.geom.assign(nall * 16, 0.0f);
    out.index.assign(nall * 4, -1);
    out.bound.assign(ng / 2 * 16, 0.0f);
    out.node.assign(ng / kNodeGroups / 2 * 16, 0.0f);
    for (size_t gi = 0; gi < nall; gi++) {
        const Group& g = gi < nbig ? bigg[gi] : groups[gi - nbig];
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
    }
    auto members_of = [&](size_t g0, size_t g1) {
        std::vector<int32_t> m;
        for (size_t gi = g0; gi < std::min(g1, ng); gi++)
            for (int k = 0; k < 4; k++)
                if (groups[gi][k] >= 0) m.push_back(groups[gi][k]);
        return m;
    };
    for (size_t gi = 0; gi < ng; gi++) put_box(out.bound, gi, box_of(s, members_of(gi, gi + 1)));
    for (size_t ni = 0; ni < ng / kNodeGroups; ni++)
        put_box(out.node, ni, box_of(s, members_of(ni * kNodeGroups, (ni + 1) * kNodeGroups)));
    // top level: one box per chunk of 64 groups (the kernels' unit of work per pass)
    const size_t nt = (ng + 63) / 64, nt2 = nt + (nt & 1);
    out.top.assign(nt2 / 2 * 16, 0.0f);
    for (size_t ti = 0; ti < nt2; ti++) put_box(out.top, ti, box_of(s, members_of(ti * 64, ti * 64 + 64)));
    // the per-ray margin constants (tracer.hip, box_ray) over the hierarchy's spheres
    double rmax = 0.0, cmax = 0.0, lam = 0.0;
    for (int32_t j : normal) {
        const double r = std::fabs(static_cast<double>(s[j].radius));
        rmax = std::max(rmax, r);
        double c2 = 0.0;
        for (int a = 0; a < 3; a++) {
            const double c = s[j].center[a];
            c2 += c * c;
            lam = std::max(lam, std::fabs(c) + r);
        }
        cmax = std::max(cmax, std::sqrt(c2));
    }
    out.margin[0] = round_up(cmax * (1.0 + 1e-6));
    out.margin[1] = round_up(rmax * rmax * (1.0 + 1e-6));
    out.margin[2] = round_up(lam * (1.0 + 1e-6));
    out.margin[3] = 0.0f;
    return true;
}

}  // namespace vcrt
