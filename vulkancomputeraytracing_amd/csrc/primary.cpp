// primary.cpp -- per-tile group lists for camera rays (the flat culled scan's primary segments).
//
// A camera ray of pixel (x, y) and sample i (shader.comp:43-52) starts at the camera centre and
// points at pixel00 + (x + jx) delta_u + (y + jy) delta_v with the jitter (jx, jy) in
// [-0.5, 0.5). All camera rays of a 4x4-pixel quarter of a tile therefore lie in the pyramid
// from the centre through the quarter's footprint grown by half a pixel: the rectangle R of the
// image plane. The
// kernel evaluates that direction in fp32 (a few roundings: |error| < 1e-5 of the scene size
// here), so R is grown by a further 1e-3 world units.
//
// Which groups may such a ray need? A member with fp32 discriminant >= 0 whose root can be
// accepted (tracer.hip may_hit: hb < 0 or cc < 0) has its centre within r + M_s of the ray
// line (margin argument, tracer.hip fact (2)), and the closest line point lies at t >= 0 up to
// the rounding of hb (< 1e-5 here) or the camera lies inside the sphere. So the member's box,
// grown by the box margin M_b = K_b Q (Q = (|o| + c_max)^2 + r_max^2 with o = the camera) and
// by 1e-3, meets the pyramid. The test below keeps every box that no side plane of the pyramid
// separates from it (conservative: it ignores the other separating axes), for chunks, then
// their nodes, then their groups (a node's box and margin cover its groups' grown boxes).
// Tiles with more than kPrimaryMax groups get no list. tests/test_cull_cpu.py checks the lists
// against fp32 emulations of the kernel's camera rays and discriminants.
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <limits>
#include <thread>

#include "cluster.hpp"
#include "vcrt_math.h"

namespace vcrt {
namespace {

struct DBox {
    double c[3], h[3];  // centre, half extent (grown)
    bool always = false;
};

// Element i of a pair-SoA box table, grown by its margin K * Q and `extra`.
DBox grown_box(const std::vector<float>& table, size_t i, double Q, double extra) {
    const float* t = &table[(i / 2) * 16];
    const int e = static_cast<int>(i % 2);
    DBox b;
    const double K = t[12 + e];
    const double g = K * Q * (1.0 + 1e-6) + extra;
    b.always = !(g < 1e30);  // K = inf: a zero radius, never ruled out
    for (int a = 0; a < 3; a++) {
        const double lo = t[2 * a + e], hi = t[6 + 2 * a + e];
        b.c[a] = 0.5 * (lo + hi);
        b.h[a] = 0.5 * (hi - lo) + g;
    }
    return b;
}

struct Pyramid {
    double apex[3];
    double n[4][3];  // inward side-plane normals
};

// No side plane separates the sphere (centre c, radius R) from the pyramid (conservative).
bool sphere_outside(const Pyramid& P, const double c[3], double R) {
    for (int k = 0; k < 4; k++) {
        double s = 0.0, nn = 0.0;
        for (int a = 0; a < 3; a++) {
            s += P.n[k][a] * (c[a] - P.apex[a]);
            nn += P.n[k][a] * P.n[k][a];
        }
        if (s + std::sqrt(nn) * R < 0.0) return true;
    }
    return false;
}

bool outside(const Pyramid& P, const DBox& b) {
    if (b.always) return false;
    for (int k = 0; k < 4; k++) {
        double s = 0.0, r = 0.0;
        for (int a = 0; a < 3; a++) {
            s += P.n[k][a] * (b.c[a] - P.apex[a]);
            r += std::fabs(P.n[k][a]) * b.h[a];
        }
        if (s + r < 0.0) return true;
    }
    return false;
}

}  // namespace

namespace {

// The quarters of a rank's local tiles and, per quarter, the pyramid of its camera rays and the
// hierarchy groups whose grown boxes it may meet (chunks, then their nodes, then their groups).
struct QuarterWalker {
    const CullTables& ct;
    double p00[3], du[3], dv[3], o[3];
    double ndu, ndv, Q;
    uint32_t tiles_x, nloc;
    int32_t rank, world;
    std::vector<DBox> gb, nb, tb;
    std::vector<bool> real;
    static constexpr double kExtra = 1e-3;

    QuarterWalker(const CullTables& c, const float cam[12], int32_t width, int32_t height,
                  int32_t r, int32_t w)
        : ct(c), rank(r), world(w) {
        tiles_x = static_cast<uint32_t>((width + 7) / 8);
        const uint32_t tiles_y = static_cast<uint32_t>((height + 7) / 8);
        for (int a = 0; a < 3; a++) {
            p00[a] = cam[a];
            du[a] = cam[3 + a];
            dv[a] = cam[6 + a];
            o[a] = cam[9 + a];
        }
        const double on = std::sqrt(o[0] * o[0] + o[1] * o[1] + o[2] * o[2]);
        Q = (on + ct.margin[0]) * (on + ct.margin[0]) + ct.margin[1];
        ndu = std::sqrt(du[0] * du[0] + du[1] * du[1] + du[2] * du[2]);
        ndv = std::sqrt(dv[0] * dv[0] + dv[1] * dv[1] + dv[2] * dv[2]);
        const size_t ng = static_cast<size_t>(ct.ngroups);
        gb.resize(ng);
        nb.resize(ng / kNodeGroups);
        tb.resize((ng + 63) / 64);
        for (size_t i = 0; i < gb.size(); i++) gb[i] = grown_box(ct.bound, i, Q, kExtra);
        for (size_t i = 0; i < nb.size(); i++) nb[i] = grown_box(ct.node, i, Q, kExtra);
        for (size_t i = 0; i < tb.size(); i++) tb[i] = grown_box(ct.top, i, Q, kExtra);
        real.assign(ng, false);
        for (size_t i = 0; i < ng; i++)
            for (int k = 0; k < 4; k++) real[i] = real[i] || ct.index[(ct.nbig + i) * 4 + k] >= 0;
        // local tiles in the kernel's order (vcrt_math.h tile_of)
        nloc = 0;
        for (uint32_t ty = 0; ty < tiles_y; ty++)
            for (uint32_t tx = 0; tx < tiles_x; tx++)
                if ((tx + ty) % static_cast<uint32_t>(world) == static_cast<uint32_t>(rank)) nloc++;
    }

    // entry e = 4 lt + 2 qy + qx: the 4x4-pixel quarter (qx, qy) of local tile lt
    Pyramid pyramid(uint32_t e) const {
        const uint32_t lt = e >> 2, qx = e & 1u, qy = (e >> 1) & 1u;
        uint32_t tx, ty;
        tile_of(lt, static_cast<uint32_t>(rank), static_cast<uint32_t>(world), tiles_x, &tx, &ty);
        // the footprint of the quarter's sample points, grown by kExtra in the image plane
        const double x0 = 8.0 * tx + 4.0 * qx, y0 = 8.0 * ty + 4.0 * qy;
        const double X0 = x0 - 0.5 - kExtra / ndu, X1 = x0 + 3.5 + kExtra / ndu;
        const double Y0 = y0 - 0.5 - kExtra / ndv, Y1 = y0 + 3.5 + kExtra / ndv;
        const double XY[4][2] = {{X0, Y0}, {X1, Y0}, {X1, Y1}, {X0, Y1}};
        double D[4][3], mid[3] = {0, 0, 0};
        for (int k = 0; k < 4; k++)
            for (int a = 0; a < 3; a++) {
                D[k][a] = p00[a] + XY[k][0] * du[a] + XY[k][1] * dv[a] - o[a];
                mid[a] += 0.25 * D[k][a];
            }
        Pyramid P;
        for (int a = 0; a < 3; a++) P.apex[a] = o[a];
        for (int k = 0; k < 4; k++) {
            const double* u = D[k];
            const double* v = D[(k + 1) % 4];
            double n[3] = {u[1] * v[2] - u[2] * v[1], u[2] * v[0] - u[0] * v[2],
                           u[0] * v[1] - u[1] * v[0]};
            const double s = n[0] * mid[0] + n[1] * mid[1] + n[2] * mid[2];
            for (int a = 0; a < 3; a++) P.n[k][a] = s < 0.0 ? -n[a] : n[a];
        }
        return P;
    }

    // The groups the pyramid may meet, in hierarchy order; false when there are more than `cap`.
    bool groups(const Pyramid& P, uint32_t cap, std::vector<uint32_t>& found) const {
        found.clear();
        for (size_t ci = 0; ci < tb.size(); ci++) {
            if (outside(P, tb[ci])) continue;
            for (size_t ni = ci * 8; ni < std::min(nb.size(), ci * 8 + 8); ni++) {
                if (outside(P, nb[ni])) continue;
                for (size_t gi = ni * kNodeGroups; gi < ni * kNodeGroups + kNodeGroups; gi++) {
                    if (!real[gi] || outside(P, gb[gi])) continue;
                    if (found.size() == cap) return false;
                    found.push_back(static_cast<uint32_t>(gi));
                }
            }
        }
        return true;
    }
};

// Runs body(begin, end, part) over [0, n) in contiguous parts on up to 16 host threads
// (VCRT_HOST_THREADS overrides; parts of at least 2048 quarters); part p covers a range after
// part p - 1's, so concatenating per-part outputs in part order gives the serial result.
template <typename Body>
uint32_t parallel_parts(uint32_t n, Body&& body) {
    uint32_t threads = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
    if (const char* e = std::getenv("VCRT_HOST_THREADS"))
        threads = static_cast<uint32_t>(std::min(16, std::max(1, std::atoi(e))));
    const uint32_t parts = std::max(1u, std::min(threads, (n + 2047) / 2048));
    const uint32_t per = (n + parts - 1) / parts;
    std::vector<std::thread> pool;
    for (uint32_t t = 1; t < parts; t++)
        pool.emplace_back([&, t] { body(std::min(n, t * per), std::min(n, (t + 1) * per), t); });
    body(0, std::min(n, per), 0u);
    for (auto& th : pool) th.join();
    return parts;
}

}  // namespace

void build_primary_lists(const CullTables& ct, const float cam[12], int32_t width,
                         int32_t height, int32_t rank, int32_t world, PrimaryLists& out) {
    out.info.clear();
    out.ids.clear();
    const QuarterWalker qw(ct, cam, width, height, rank, world);
    const size_t ng = static_cast<size_t>(ct.ngroups);
    const uint32_t n = 4 * qw.nloc;
    out.info.assign(n, kPrimaryNone);
    // per part: its quarters' group ids, offsets relative to the part (fixed up below)
    std::vector<std::vector<uint16_t>> ids(16);
    const uint32_t parts = parallel_parts(n, [&](uint32_t b, uint32_t e_end, uint32_t part) {
        std::vector<uint32_t> found;
        std::vector<uint16_t>& mine = ids[part];
        for (uint32_t e = b; e < e_end; e++) {
            const bool fits = qw.groups(qw.pyramid(e), kPrimaryMax, found);
            const size_t cnt = found.size();
            if (!fits || ng > 0xFFFFu) continue;  // ids are uint16
            out.info[e] = static_cast<uint32_t>(mine.size()) << 4 | static_cast<uint32_t>(cnt);
            for (uint32_t g : found) mine.push_back(static_cast<uint16_t>(g));
        }
    });
    // concatenate in part order; offsets are 28-bit: beyond that a quarter keeps no list
    const uint32_t per = (n + parts - 1) / parts;
    for (uint32_t part = 0; part < parts; part++) {
        const size_t base = out.ids.size();
        for (uint32_t e = part * per; e < std::min(n, (part + 1) * per); e++) {
            if (out.info[e] == kPrimaryNone) continue;
            const size_t off = base + (out.info[e] >> 4);
            out.info[e] = off + (out.info[e] & 15u) >= (size_t{1} << 28)
                              ? kPrimaryNone
                              : static_cast<uint32_t>(off) << 4 | (out.info[e] & 15u);
        }
        out.ids.insert(out.ids.end(), ids[part].begin(), ids[part].end());
    }
}

void build_primary_sphere_lists(const CullTables& ct, const vcrt_sphere* spheres,
                                const float cam[12], int32_t width, int32_t height, int32_t rank,
                                int32_t world, PrimarySphereLists& out) {
    out.info.clear();
    out.rec.clear();
    const QuarterWalker qw(ct, cam, width, height, rank, world);
    const uint32_t n = 4 * qw.nloc;
    out.info.assign(n, kPrimaryNone);
    const float ox = cam[9], oy = cam[10], oz = cam[11];
    // per part: its quarters' pair records, first pair relative to the part (fixed up below)
    std::vector<std::vector<float>> recs(16);
    const uint32_t parts = parallel_parts(n, [&](uint32_t b, uint32_t e_end, uint32_t part) {
        std::vector<uint32_t> found;
        std::vector<int32_t> members;
        std::vector<float>& mine = recs[part];
        for (uint32_t e = b; e < e_end; e++) {
            const Pyramid P = qw.pyramid(e);
            // the group walk bounds the work; a quarter meeting very many groups keeps no list
            if (!qw.groups(P, 64, found)) continue;
            members.clear();
            bool over = false;
            for (uint32_t gi : found) {
                for (int k = 0; k < 4 && !over; k++) {
                    const int32_t j = ct.index[(ct.nbig + gi) * 4 + k];
                    if (j < 0) continue;
                    const vcrt_sphere& sp = spheres[j];
                    const double c[3] = {sp.center[0], sp.center[1], sp.center[2]};
                    const double r = std::fabs(static_cast<double>(sp.radius));
                    double oc2 = 0.0;
                    for (int a = 0; a < 3; a++) oc2 += (qw.o[a] - c[a]) * (qw.o[a] - c[a]);
                    // the member's own margin (tracer.hip fact (2)), and the rounding of the rays
                    const double Ms = r > 0.0 ? 8.1 * 0x1p-24 * (oc2 + r * r) / r * (1.0 + 1e-5)
                                              : std::numeric_limits<double>::infinity();
                    if (!(Ms < 1e30) || !sphere_outside(P, c, r + Ms + QuarterWalker::kExtra)) {
                        if (members.size() == kPrimarySphereMax) over = true;
                        else members.push_back(j);
                    }
                }
            }
            if (over) continue;
            out.info[e] = static_cast<uint32_t>(mine.size() / 12) << 4 |
                          static_cast<uint32_t>(members.size());
            for (size_t m = 0; m < members.size(); m += 2) {
                float r[12] = {0, 0, 0, 0, 0, 0, 3.0e38f, 3.0e38f, 0, 0, 0, 0};
                int32_t idx[2] = {-1, -1};
                for (int e2 = 0; e2 < 2 && m + e2 < members.size(); e2++) {
                    const vcrt_sphere& sp = spheres[members[m + e2]];
                    // pair_disc_cc's operations and order: oc = o - c, cc = ((ocx ocx + ocy ocy)
                    // + ocz ocz) - r^2 with r^2 = radius * radius, fp32, no FMA
                    const float ocx = ox - sp.center[0], ocy = oy - sp.center[1],
                                ocz = oz - sp.center[2];
                    const float r2 = sp.radius * sp.radius;
                    r[0 + e2] = ocx;
                    r[2 + e2] = ocy;
                    r[4 + e2] = ocz;
                    r[6 + e2] = ((ocx * ocx + ocy * ocy) + ocz * ocz) - r2;
                    idx[e2] = members[m + e2];
                }
                std::memcpy(&r[8], idx, sizeof(idx));
                mine.insert(mine.end(), r, r + 12);
            }
        }
    });
    // concatenate in part order; first pairs are 28-bit: beyond that a quarter keeps no list
    const uint32_t per = (n + parts - 1) / parts;
    for (uint32_t part = 0; part < parts; part++) {
        const size_t base = out.rec.size() / 12;
        for (uint32_t e = part * per; e < std::min(n, (part + 1) * per); e++) {
            if (out.info[e] == kPrimaryNone) continue;
            const size_t first = base + (out.info[e] >> 4);
            out.info[e] = first >= (size_t{1} << 28)
                              ? kPrimaryNone
                              : static_cast<uint32_t>(first) << 4 | (out.info[e] & 15u);
        }
        out.rec.insert(out.rec.end(), recs[part].begin(), recs[part].end());
    }
}

void build_camera_records(const CullTables& ct, const float cam[12], std::vector<float>& out) {
    const size_t nall = static_cast<size_t>(ct.nbig + ct.ngroups);
    out.assign(nall * 16, 0.0f);
    const float ox = cam[9], oy = cam[10], oz = cam[11];
    for (size_t gi = 0; gi < nall; gi++) {
        const float* g = &ct.geom[gi * 16];
        float* c = &out[gi * 16];
        for (int pair = 0; pair < 2; pair++)
            for (int e = 0; e < 2; e++) {
                // pair-SoA: (cx0,cx1,cy0,cy1) (cz0,cz1,r0^2,r1^2) per pair of members
                const float* q = g + 8 * pair;
                float* w = c + 8 * pair;
                const float ocx = ox - q[0 + e], ocy = oy - q[2 + e], ocz = oz - q[4 + e];
                // pair_disc_cc's order: ((ocx ocx + ocy ocy) + ocz ocz) - r^2, fp32, no FMA
                const float cc = ((ocx * ocx + ocy * ocy) + ocz * ocz) - q[6 + e];
                w[0 + e] = ocx;
                w[2 + e] = ocy;
                w[4 + e] = ocz;
                w[6 + e] = cc;
            }
    }
}

}  // namespace vcrt
