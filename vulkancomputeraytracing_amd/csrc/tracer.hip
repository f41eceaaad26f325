// tracer.hip -- the hot path: per-pixel ray generation -> sphere-list intersection ->
// Lambertian / metal / glass scatter -> multi-bounce radiance accumulation, written for
// gfx950 (CDNA4, wave64) as a persistent-lanes wavefront tracer.
//
// Reference semantics (quirks kept):
//   shaders/shader.comp:16-58            camera ray per sample, accumulate, divide, store
//   shaders/include/functions.glsl:14-40 hit_sphere (strict <, index-order tie break)
//   shaders/include/functions.glsl:65-92 ray_color bounce loop, sky on miss
//   shaders/include/textures.glsl:19-71  lambertian / metal / glass scatter
//
// MI355X design:
//   * Work items are (8x8 pixel tile, chunk of K samples, slot): one lane per pixel, the
//     chunk's samples in order. A wave takes a whole block (one tile at one chunk = 64 items)
//     with one atomic and hands its slots to lanes as they free up; a lane whose path ends
//     starts its next sample at once (path regeneration). Chunk sums go to a [chunk][pixel]
//     slab in HBM and vcrt_resolve adds them in chunk order (K >= spp: no slab, the
//     reference's sequential sum).
//   * Ray state lives in VGPRs. Sphere tests run two spheres per packed-fp32 instruction
//     (v_pk_add_f32 / v_pk_mul_f32 on pair-SoA groups of four: 2 lane-ops per issue, the only
//     way gfx950 reaches its fp32 peak).
//   * The sphere-list scan is either the reference's linear scan (wave-uniform groups through
//     the scalar cache or LDS) or an exact culled scan over a spatial hierarchy (groups of 4,
//     nodes of 8 groups, chunks of 64 groups), wave-uniform or per lane on an LDS copy of the
//     tables; see "Culled scan" below for why it returns the same sphere and t.
//   * Only fp32 add/sub/mul plus correctly rounded div/sqrt, no contraction, in everything
//     that reaches the image: results are bit-identical to the CPU oracle for the same
//     accumulation order. No MFMA.
#include <hip/hip_runtime.h>

#include "vcrt_kernel_abi.h"
#include "vcrt_math.h"

#pragma clang fp contract(off)

using namespace vcrt;

namespace {

typedef float v2f __attribute__((ext_vector_type(2)));

__device__ __forceinline__ uint32_t lanes_below(uint64_t mask) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32),
                                     __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u));
}

typedef __attribute__((address_space(4))) const float4 cfloat4;

// One group = four spheres in pair-SoA form: q[0] = (cx0,cx1,cy0,cy1), q[1] = (cz0,cz1,r0²,r1²),
// q[2] = (cx2,cx3,cy2,cy3), q[3] = (cz2,cz3,r2²,r3²).
struct Group {
    float4 q[4];
};

template <bool kLds>
__device__ __forceinline__ Group load_group(const float4* lds, const TraceParams& p, int gi) {
    Group g;
    if constexpr (kLds) {
#pragma unroll
        for (int k = 0; k < 4; ++k) g.q[k] = lds[4 * gi + k];
    } else {
        cfloat4* s = (cfloat4*)p.geom;  // wave-uniform index -> s_load through the scalar cache
#pragma unroll
        for (int k = 0; k < 4; ++k) g.q[k] = s[4 * gi + k];
    }
    return g;
}

// hit_sphere (functions.glsl:14-40) after the discriminant test passed: nearest root in
// (min_t, max_t), strict comparisons, max_t shrinks on acceptance.
__device__ __forceinline__ void accept_root(float hb, float disc, float a, float& max_t, int& best,
                                            int j) {
    const float min_t = 0.001f;
    const float sq = __builtin_sqrtf(disc);
    float root = (-hb - sq) / a;
    bool ok = true;
    if (root <= min_t || max_t <= root) {
        root = (-hb + sq) / a;
        ok = !(root <= min_t || max_t <= root);
    }
    if (ok) {
        max_t = root;
        best = j;
    }
}

// Conservative pre-filter for the root path: false only when hit_sphere would certainly reject
// the sphere, decided without the correctly rounded sqrt/divisions.
//   sq_hi >= RN(sqrt(disc)): hardware v_sqrt_f32 (~1 ulp) plus 4 ulp;
//   x1_lo = RN(-hb - sq_hi) <= x1 and x2_hi = RN(-hb + sq_hi) >= x2 (rounding is monotone);
//   "beyond": x1_lo - max_t*a >= 0 (the sign of the fused fma is exact: every operand is a
//   multiple of >= 2^-76 in the guarded ranges, so nothing underflows) => x1/a >= max_t =>
//   root1 = RN(x1/a) >= max_t and root2 >= root1: both rejected;
//   "behind": x2_hi - min_t*a <= 0 => root2 <= min_t and root1 <= root2: both rejected.
// Outside the guarded ranges (tiny/huge/NaN values) it answers true and the exact path decides.
__device__ __forceinline__ bool may_accept(float hb, float disc, float a, float max_t,
                                           bool ray_ok) {
    const float min_t = 0.001f;
    const bool ok = ray_ok && disc >= 0x1p-100f && disc <= 0x1p100f && hb >= -0x1p60f &&
                    hb <= 0x1p60f;
    const float sq_hi = __uint_as_float(__float_as_uint(__builtin_amdgcn_sqrtf(disc)) + 4u);
    const float x1_lo = -hb - sq_hi;
    const float x2_hi = -hb + sq_hi;
    const bool beyond = __builtin_fmaf(-max_t, a, x1_lo) >= 0.0f;
    const bool behind = __builtin_fmaf(-min_t, a, x2_hi) <= 0.0f;
    return !ok || !(beyond || behind);
}

// Discriminants of two spheres at once (hit_sphere's first half, element-wise exact):
// oc = o - c; half_b = dot(oc, d); c = dot(oc, oc) - r²; disc = half_b² - a·c.
__device__ __forceinline__ void pair_disc(const v2f ox, const v2f oy, const v2f oz, const v2f dx,
                                          const v2f dy, const v2f dz, const v2f a2, float4 xy,
                                          float4 zr, v2f& hb, v2f& disc) {
    const v2f cx = {xy.x, xy.y}, cy = {xy.z, xy.w}, cz = {zr.x, zr.y}, r2 = {zr.z, zr.w};
    const v2f ocx = ox - cx, ocy = oy - cy, ocz = oz - cz;
    hb = ocx * dx + ocy * dy + ocz * dz;
    const v2f cc = (ocx * ocx + ocy * ocy + ocz * ocz) - r2;
    disc = hb * hb - a2 * cc;
}

// The sphere-list scan of one ray segment (functions.glsl:77-81): four spheres per step as two
// packed pairs, the next group prefetched, one wave-uniform branch into the rare root path,
// which then visits the four candidates in index order so ties resolve to the earlier sphere.
template <bool kLds>
__device__ __forceinline__ void scan_spheres(const TraceParams& p, const float4* lds, int n,
                                             const f3 o, const f3 d, float& max_t, int& best,
                                             uint32_t& hit_groups) {
    const float a = dot(d, d);  // loop-invariant in hit_sphere: hoisting is exact
    // the pre-filter's guarded range: a in [2^-20, 2^60] (and not NaN)
    const bool ray_ok = a >= 0x1p-20f && a <= 0x1p60f;
    // |o| <= 2^30 and a <= 2^60 (|d| <= 2^30) with the host-checked scene bound |c|, r <= 2^30
    // keep every discriminant finite (hb^2, a*c < 2^127): no NaN can reach the max test
    const bool finite_ok = (p.flags & kFlagSceneBounded) != 0 && a <= 0x1p60f &&
                           fabsf(o.x) <= 0x1p30f && fabsf(o.y) <= 0x1p30f &&
                           fabsf(o.z) <= 0x1p30f;
    const uint64_t unguarded = __ballot(!finite_ok);
    const v2f ox = {o.x, o.x}, oy = {o.y, o.y}, oz = {o.z, o.z};
    const v2f dx = {d.x, d.x}, dy = {d.y, d.y}, dz = {d.z, d.z}, a2 = {a, a};
    const int ngroups = (n + 3) >> 2;
    Group g = load_group<kLds>(lds, p, 0);
    for (int gi = 0; gi < ngroups; ++gi) {
        const Group nx = load_group<kLds>(lds, p, gi + 1);  // table padded by one group
        v2f hb01, d01, hb23, d23;
        pair_disc(ox, oy, oz, dx, dy, dz, a2, g.q[0], g.q[1], hb01, d01);
        pair_disc(ox, oy, oz, dx, dy, dz, a2, g.q[2], g.q[3], hb23, d23);
        // Any of the four not negative? For finite discriminants this is !(max < 0): one
        // v_max3 + v_max + compare instead of four compares. Lanes whose ray is outside the
        // guarded range (where a discriminant could be NaN, which max would drop) always take
        // the exact per-sphere test below.
        const float m4 = fmaxf(fmaxf(d01.x, d01.y), fmaxf(d23.x, d23.y));
        if (__ballot(!(m4 < 0.0f)) | unguarded) {
            const bool h0 = !(d01.x < 0.0f), h1 = !(d01.y < 0.0f), h2 = !(d23.x < 0.0f),
                       h3 = !(d23.y < 0.0f);
            ++hit_groups;
            const int j = 4 * gi;  // padding spheres (index >= n) are never accepted
            // pre-filter against the max_t at group entry: a rejection stays valid as max_t
            // only shrinks; survivors go through hit_sphere's exact logic in index order
            const float mt = max_t;
            const bool e0 = h0 && may_accept(hb01.x, d01.x, a, mt, ray_ok);
            const bool e1 = h1 && j + 1 < n && may_accept(hb01.y, d01.y, a, mt, ray_ok);
            const bool e2 = h2 && j + 2 < n && may_accept(hb23.x, d23.x, a, mt, ray_ok);
            const bool e3 = h3 && j + 3 < n && may_accept(hb23.y, d23.y, a, mt, ray_ok);
            if (__ballot(e0) | __ballot(e1) | __ballot(e2) | __ballot(e3)) {
                if (e0) accept_root(hb01.x, d01.x, a, max_t, best, j + 0);
                if (e1) accept_root(hb01.y, d01.y, a, max_t, best, j + 1);
                if (e2) accept_root(hb23.x, d23.x, a, max_t, best, j + 2);
                if (e3) accept_root(hb23.y, d23.y, a, max_t, best, j + 3);
            }
        }
        g = nx;
    }
}

// ---------------------------------------------------------------------------------------------
// Culled scan (variant CULL). Exact for waves whose rays are all in the guarded finite range
// (|o| <= 2^30, a in [2^-20, 2^60], scene bounded), by two facts:
//  (1) hit_sphere's sequential scan with strict < (functions.glsl:27-29,77-81) selects the
//      candidate with the smallest t, earliest index on ties, where t = root1 if root1 > min_t
//      else root2, kept if min_t < t < max_t -- so spheres may be visited in any order;
//  (2) a margin. With u = 2^-24, disc_f >= 0 (pair_disc's rounded oc, hb, cc, products and
//      difference) implies that the ray line passes within r + M_s of the centre,
//      M_s = 8.1u (|oc|^2 + r^2) / r: the roundings move hb^2 - a*cc by at most ~15u a |oc|^2
//      and the rounded oc moves the centre by u |oc|. For a bound (C, R) of members with
//      radius >= r_min, |oc|^2 + r^2 <= 2 |oC|^2 + 3 R^2, so M = Kc (|oC|^2 + 1.5 R^2) with
//      Kc = 32.4u / r_min covers every member twice over.
// Bound test, per lane: with the approximate unit direction w = d * rsq(a) (|w| = 1 + O(10u))
// and h = (o - C).w, X = |oC|^2 - h^2 approximates the squared line distance within 35u |oC|^2
// (rounded oc, w, h, |oC|^2, X). The lane rules the bound out when X > RM^2 with
//   RM = K |oC|^2 + Rk,  K = Kc (1 + 1e-5) + 6e-6 / (2R),  Rk = (R + 1.5 Kc R^2)(1 + 1e-5)
// (host constants, rounded up), since RM^2 >= (R + M)^2 (1 + 2e-5) + 6e-6 |oC|^2 and 6e-6 > 35u:
// the line then misses every member by more than its margin, so no member has disc_f >= 0.
// Waves holding a ray outside the guarded range scan the original table in reference order.

// t of one candidate as hit_sphere would accept it (finite case, fact (1)).
__device__ __forceinline__ float candidate_t(float hb, float disc, float a) {
    const float sq = __builtin_sqrtf(disc);
    const float r1 = (-hb - sq) / a;
    if (r1 > 0.001f) return r1;
    return (-hb + sq) / a;
}

// A member whose origin lies outside or on it (cc >= 0) while the ray points away from its
// centre (hb >= 0) can never be accepted: disc_f <= RN(hb^2) and RN(sqrt(RN(hb^2))) = hb
// (binary fp, no underflow), so RN(-hb + sq) <= 0 and both roots are <= 0 < min_t. If hb^2
// underflows (hb < 2^-63), RN(hb^2) is off by at most 2^-149, so -hb + sq < 2^-74 and, with
// a >= 2^-20, root2 < 2^-54 < min_t all the same.
// A -0 hb only adds candidates; cc is never -0. (Padding members never hit: their
// r^2 = -3e38 makes disc negative or -inf.)
__device__ __forceinline__ bool may_hit(float hb, float cc, float disc) {
    return !(disc < 0.0f) && (hb < 0.0f || cc < 0.0f);
}

// pair_disc that also returns cc = |oc|^2 - r^2 (for may_hit).
__device__ __forceinline__ void pair_disc_cc(const v2f ox, const v2f oy, const v2f oz,
                                             const v2f dx, const v2f dy, const v2f dz,
                                             const v2f a2, float4 xy, float4 zr, v2f& hb,
                                             v2f& cc, v2f& disc) {
    const v2f cx = {xy.x, xy.y}, cy = {xy.z, xy.w}, cz = {zr.x, zr.y}, r2 = {zr.z, zr.w};
    const v2f ocx = ox - cx, ocy = oy - cy, ocz = oz - cz;
    hb = ocx * dx + ocy * dy + ocz * dz;
    cc = (ocx * ocx + ocy * ocy + ocz * ocz) - r2;
    disc = hb * hb - a2 * cc;
}

__device__ __forceinline__ void consider(float t, int idx, float& max_t, int& best) {
    if (t > 0.001f && (t < max_t || (t == max_t && best >= 0 && idx < best))) {
        max_t = t;
        best = idx;
    }
}

__device__ __forceinline__ v2f vfma(v2f x, v2f y, v2f z) {
    return __builtin_elementwise_fma(x, y, z);
}

// 1 when the wave-uniform x != 0, in SALU (the compiler lowers `x ? 1 : 0` of a ballot
// result through a VGPR: v_cndmask + v_readfirstlane per test).
__device__ __forceinline__ uint32_t nonzero(uint64_t x) {
    uint32_t r;
    asm volatile("s_cmp_lg_u64 %1, 0\n\ts_cselect_b32 %0, 1, 0" : "=s"(r) : "s"(x) : "scc");
    return r;
}

struct CullRay {  // one ray, splatted for packed tests
    v2f ox, oy, oz;  // origin
    v2f wx, wy, wz;  // approximate unit direction
};

// Bound test of one pair (TraceParams.cbound: (Cx0,Cx1,Cy0,Cy1) (Cz0,Cz1,K0,K1)
// (Rk0,Rk1,-,-)): bit 0/1 set when some lane may accept a member of bound 0/1 (NaN compares as
// "may").
struct BoundPair {
    float4 b0, b1;
    float2 b2;
};

__device__ __forceinline__ BoundPair load_bound_pair(cfloat4* b) {
    return BoundPair{b[0], b[1], *(__attribute__((address_space(4))) const float2*)(b + 2)};
}

template <bool kStats>
__device__ __forceinline__ uint32_t bound_pair_need(const CullRay& r, const BoundPair& bp,
                                                    uint32_t& lane_needs, uint32_t& lane_cnt) {
    const float4 b0 = bp.b0, b1 = bp.b1;
    const float2 b2 = bp.b2;
    const v2f Cx = {b0.x, b0.y}, Cy = {b0.z, b0.w}, Cz = {b1.x, b1.y};
    const v2f K = {b1.z, b1.w}, Rk = {b2.x, b2.y};
    const v2f ocx = r.ox - Cx, ocy = r.oy - Cy, ocz = r.oz - Cz;
    const v2f oc2 = vfma(ocz, ocz, vfma(ocy, ocy, ocx * ocx));
    const v2f h = vfma(ocz, r.wz, vfma(ocy, r.wy, ocx * r.wx));
    const v2f X = vfma(-h, h, oc2);   // ~ squared line distance
    const v2f RM = vfma(K, oc2, Rk);  // >= R + M, with the slack folded in
    const v2f T = RM * RM;
    const uint64_t n0 = __ballot(!(X.x > T.x)), n1 = __ballot(!(X.y > T.y));
    if constexpr (kStats) {
        lane_needs += __popcll(n0) + __popcll(n1);
        lane_cnt += (uint32_t)!(X.x > T.x) + (uint32_t)!(X.y > T.y);
    }
    return nonzero(n0) | (nonzero(n1) << 1);
}

// The exact test of one group for every lane (wave-uniform scalar loads of the 80-B record):
// the big-sphere list, tested for every ray ahead of the hierarchy.
__device__ __forceinline__ void exact_group_uniform(cfloat4* rec, const CullRay& r, v2f dx, v2f dy,
                                                    v2f dz, v2f a2, float a, float& max_t,
                                                    int& best) {
    const float4 q0 = rec[0], q1 = rec[1], q2 = rec[2], q3 = rec[3];
    v2f hb01, cc01, d01, hb23, cc23, d23;
    pair_disc_cc(r.ox, r.oy, r.oz, dx, dy, dz, a2, q0, q1, hb01, cc01, d01);
    pair_disc_cc(r.ox, r.oy, r.oz, dx, dy, dz, a2, q2, q3, hb23, cc23, d23);
    const float m4 = fmaxf(fmaxf(d01.x, d01.y), fmaxf(d23.x, d23.y));
    if (__ballot(!(m4 < 0.0f))) {
        const float4 idf = rec[4];
        if (may_hit(hb01.x, cc01.x, d01.x))
            consider(candidate_t(hb01.x, d01.x, a), __float_as_int(idf.x), max_t, best);
        if (may_hit(hb01.y, cc01.y, d01.y))
            consider(candidate_t(hb01.y, d01.y, a), __float_as_int(idf.y), max_t, best);
        if (may_hit(hb23.x, cc23.x, d23.x))
            consider(candidate_t(hb23.x, d23.x, a), __float_as_int(idf.z), max_t, best);
        if (may_hit(hb23.y, cc23.y, d23.y))
            consider(candidate_t(hb23.y, d23.y, a), __float_as_int(idf.w), max_t, best);
    }
}

// Stats builds count in `hit_groups` the lanes that need each group (sum over group bounds)
// and in `lane_cnt` the groups this lane needs.
template <bool kStats>
__device__ __forceinline__ void scan_culled(const TraceParams& p, const f3 o, const f3 d,
                                            float& max_t, int& best, uint64_t& groups_tested,
                                            uint64_t& bounds_tested, uint32_t& hit_groups,
                                            uint32_t& lane_cnt) {
    uint32_t node_lanes = 0, node_cnt = 0;
    const float a = dot(d, d);
    const float inv = __builtin_amdgcn_rsqf(a);
    CullRay r;
    r.ox = (v2f){o.x, o.x};
    r.oy = (v2f){o.y, o.y};
    r.oz = (v2f){o.z, o.z};
    r.wx = (v2f){d.x * inv, d.x * inv};
    r.wy = (v2f){d.y * inv, d.y * inv};
    r.wz = (v2f){d.z * inv, d.z * inv};
    const v2f dx = {d.x, d.x}, dy = {d.y, d.y}, dz = {d.z, d.z}, a2 = {a, a};
    cfloat4* bound = (cfloat4*)p.cbound;
    cfloat4* node = (cfloat4*)p.cnode;
    cfloat4* geom = (cfloat4*)p.cgroup;
    for (int gb = 0; gb < p.nbig; ++gb)  // the big spheres, for every ray
        exact_group_uniform(geom + 5 * gb, r, dx, dy, dz, a2, a, max_t, best);
    groups_tested += (uint64_t)p.nbig;
    geom += 5 * p.nbig;           // the hierarchy's groups
    const int ncg = p.ncgroups;  // multiple of 16: whole node pairs
    cfloat4* top = (cfloat4*)p.ctop;
    uint32_t tops = 0;
    for (int base = 0; base < ncg; base += 64) {
        // level 0: the chunk's own bound (tested for two chunks at a time)
        if ((base & 127) == 0) {
            tops = bound_pair_need<false>(r, load_bound_pair(top + 3 * (base >> 7)), node_lanes,
                                          node_cnt);
            bounds_tested += 2;
        }
        if (((tops >> ((base >> 6) & 1)) & 1u) == 0) continue;
        // level 1: which of the next (up to) 8 nodes of 8 groups may any lane hit? (the
        // scalar loads run one pair ahead of the tests)
        const int nn = min(8, (ncg - base) >> 3);
        cfloat4* nb = node + 3 * (base >> 4);
        uint32_t nodes = 0;
        BoundPair cur = load_bound_pair(nb);
        for (int j = 0; j < nn; j += 2) {
            const BoundPair nxt = load_bound_pair(nb + 3 * ((j + 2 < nn ? j + 2 : j) >> 1));
            nodes |= bound_pair_need<false>(r, cur, node_lanes, node_cnt) << j;
            cur = nxt;
        }
        bounds_tested += (uint64_t)(nn + 8 * __popc(nodes));
        // level 2: which groups of those nodes?
        uint64_t need = 0;
        if (nodes) cur = load_bound_pair(bound + 3 * ((base + 8 * __builtin_ctz(nodes)) >> 1));
        while (nodes) {
            const int j = __builtin_ctz(nodes);
            nodes &= nodes - 1;
            cfloat4* gb = bound + 3 * ((base + 8 * j) >> 1);
            cfloat4* gnext = bound + 3 * ((base + 8 * (nodes ? __builtin_ctz(nodes) : j)) >> 1);
#pragma unroll
            for (int k = 0; k < 8; k += 2) {
                const BoundPair nxt = load_bound_pair(k + 2 < 8 ? gb + 3 * ((k + 2) >> 1) : gnext);
                need |= (uint64_t)bound_pair_need<kStats>(r, cur, hit_groups, lane_cnt)
                        << (8 * j + k);
                cur = nxt;
            }
        }
        // the exact hit_sphere test on the groups that survived (next group prefetched)
        groups_tested += (uint64_t)__popcll(need);
        if (!need) continue;
        int gi = base + __builtin_ctzll(need);
        float4 q0 = geom[5 * gi], q1 = geom[5 * gi + 1], q2 = geom[5 * gi + 2],
               q3 = geom[5 * gi + 3];
        while (true) {
            need &= need - 1;
            const int gn = need ? base + __builtin_ctzll(need) : gi;
            const float4 n0 = geom[5 * gn], n1 = geom[5 * gn + 1], n2 = geom[5 * gn + 2],
                         n3 = geom[5 * gn + 3];
            v2f hb01, cc01, d01, hb23, cc23, d23;
            pair_disc_cc(r.ox, r.oy, r.oz, dx, dy, dz, a2, q0, q1, hb01, cc01, d01);
            pair_disc_cc(r.ox, r.oy, r.oz, dx, dy, dz, a2, q2, q3, hb23, cc23, d23);
            const float m4 = fmaxf(fmaxf(d01.x, d01.y), fmaxf(d23.x, d23.y));
            if (__ballot(!(m4 < 0.0f))) {
                const float4 idf = geom[5 * gi + 4];
                const int4 id = make_int4(__float_as_int(idf.x), __float_as_int(idf.y),
                                          __float_as_int(idf.z), __float_as_int(idf.w));
                if (may_hit(hb01.x, cc01.x, d01.x))
                    consider(candidate_t(hb01.x, d01.x, a), id.x, max_t, best);
                if (may_hit(hb01.y, cc01.y, d01.y))
                    consider(candidate_t(hb01.y, d01.y, a), id.y, max_t, best);
                if (may_hit(hb23.x, cc23.x, d23.x))
                    consider(candidate_t(hb23.x, d23.x, a), id.z, max_t, best);
                if (may_hit(hb23.y, cc23.y, d23.y))
                    consider(candidate_t(hb23.y, d23.y, a), id.w, max_t, best);
            }
            if (!need) break;
            gi = gn;
            q0 = n0;
            q1 = n1;
            q2 = n2;
            q3 = n3;
        }
    }
}

// Per-lane culled scan (variant CULL_LANE). Same tables and tests as scan_culled, but only
// the node level runs wave-uniformly (scalar loads, per-lane results); each lane then tests
// the groups of its own nodes and runs the exact test on its own groups, gathering table rows
// with per-lane addresses (from an LDS copy, or from global memory when the tables are too
// large). A wave's work becomes the largest per-lane need instead of the union over lanes.
// Lanes accept candidates with the same `consider` rule, so the result is the same.

// (acc << 1) | sign bit of v: v_alignbit_b32, one VALU per collected bit.
__device__ __forceinline__ uint32_t push_sign(uint32_t acc, float v) {
    return __builtin_amdgcn_alignbit(acc, __float_as_uint(v), 31);
}

// Sign of fma(RM, RM, -X) for both bounds of a pair: set (negative) when this lane rules the
// bound out (X > RM^2 exactly; NaN -- an infinite K at |oC| = 0 -- keeps the default NaN's
// clear sign bit, i.e. "may need"). Pushed high element first.
__device__ __forceinline__ uint32_t push_bound_pair(uint32_t acc, const CullRay& r, float4 b0,
                                                    float4 b1, float2 b2) {
    const v2f Cx = {b0.x, b0.y}, Cy = {b0.z, b0.w}, Cz = {b1.x, b1.y};
    const v2f K = {b1.z, b1.w}, Rk = {b2.x, b2.y};
    const v2f ocx = r.ox - Cx, ocy = r.oy - Cy, ocz = r.oz - Cz;
    const v2f oc2 = vfma(ocz, ocz, vfma(ocy, ocy, ocx * ocx));
    const v2f h = vfma(ocz, r.wz, vfma(ocy, r.wy, ocx * r.wx));
    const v2f X = vfma(-h, h, oc2);
    const v2f RM = vfma(K, oc2, Rk);
    const v2f D = vfma(RM, RM, -X);
    return push_sign(push_sign(acc, D.y), D.x);
}

// Sign bit set when a member may be accepted: disc >= 0 and (hb < 0 or cc < 0), by sign bits
// (a -0 hb only adds a candidate that the exact test then rejects; disc is never -0).
__device__ __forceinline__ float hit_sign(float hb, float cc, float disc) {
    return __uint_as_float((__float_as_uint(hb) | __float_as_uint(cc)) & ~__float_as_uint(disc));
}

// ---- flattened exact phase (variant CULL_FLAT) ----------------------------------------------
// The per-lane exact loop runs as many passes as the wave's busiest lane needs groups (10 when
// the mean lane needs 5). Here the wave's (lane, group) pairs are listed in LDS and dealt out
// 64 per pass, each lane testing another lane's ray (fetched with ds_bpermute); candidate roots
// are listed as well and resolved 64 at a time; every owner's (t, sphere index) minimum is kept
// in an LDS 64-bit word updated with ds_min_u64 -- the lexicographic minimum of (t, index) is
// exactly what `consider` computes, since t > 0 orders like its bit pattern.
constexpr int kPairCap = 512;   // pairs per chunk and wave (more: per-lane loop instead)
constexpr int kCandCap = 128;   // candidate roots listed before a resolve round

struct WaveScratch {
    unsigned long long key[64];  // per owner lane: (bits(t) << 32) | sphere index
    float4 cand[kCandCap];       // hb, disc, a, index | owner << 24
    uint16_t pair[kPairCap];     // owner << 6 | group within the chunk
};
static_assert(sizeof(WaveScratch) == kWaveScratchBytes, "host LDS size");

__device__ __forceinline__ unsigned long long pack_hit(float t, int idx) {
    return ((unsigned long long)__float_as_uint(t) << 32) | (uint32_t)idx;
}

// Exclusive prefix of a per-lane count c < 128 over the active lanes, and the wave total,
// from bit-sliced ballots (inactive lanes count as 0).
__device__ __forceinline__ uint32_t wave_prefix(uint32_t c, uint32_t& total) {
    uint32_t pre = 0, tot = 0;
#pragma unroll
    for (int b = 0; b < 7; ++b) {
        const uint64_t m = __ballot((c >> b) & 1u);
        pre += lanes_below(m) << b;
        tot += (uint32_t)__popcll(m) << b;
    }
    total = tot;
    return pre;
}

// Resolve the listed candidate roots, 64 per pass, into the owners' keys.
__device__ __forceinline__ void resolve_cands(WaveScratch* ws, uint32_t ncand, uint32_t rank,
                                              uint32_t nact) {
    for (uint32_t c0 = 0; c0 < ncand; c0 += nact) {
        const uint32_t j = c0 + rank;
        if (j < ncand) {
            const float4 cd = ws->cand[j];
            const float t = candidate_t(cd.x, cd.y, cd.z);
            const uint32_t w = __float_as_uint(cd.w);
            if (t > 0.001f && t < 1e5f)
                atomicMin(&ws->key[w >> 24], pack_hit(t, (int)(w & 0xFFFFFFu)));
        }
    }
}

// The exact test of this chunk's needed groups, flattened over the wave. Returns false (and
// does nothing) when the wave needs more than kPairCap pairs in this chunk.
__device__ __forceinline__ bool exact_flat(WaveScratch* ws, const float4* tg, uint64_t need,
                                           const f3 o, const f3 d, float a, uint32_t lane,
                                           uint32_t& n_passes) {
    // only the wave's live lanes run this (finished lanes are masked off): pairs and
    // candidates are dealt by rank among the live lanes, nact per pass
    const uint64_t live = __ballot(1);
    const uint32_t nact = (uint32_t)__popcll(live), rank = lanes_below(live);
    const uint32_t cnt = (uint32_t)__popcll(need);
    uint32_t total;
    const uint32_t pre = wave_prefix(cnt, total);
    if (total > (uint32_t)kPairCap) return false;
    {  // list my pairs
        uint64_t m = need;
        uint32_t pos = pre;
        while (m) {
            const uint32_t k = (uint32_t)__builtin_ctzll(m);
            m &= m - 1;
            ws->pair[pos++] = (uint16_t)((lane << 6) | k);
        }
    }
    __builtin_amdgcn_wave_barrier();
    uint32_t ncand = 0;  // wave-uniform
    for (uint32_t i0 = 0; i0 < total; i0 += nact) {
        ++n_passes;
        const uint32_t i = i0 + rank;
        const bool act = i < total;
        const uint32_t pr = act ? (uint32_t)ws->pair[i] : (lane << 6);
        const int owner = (int)(pr >> 6);
        // the owner's ray (ds_bpermute; owners are active lanes)
        const float qx = __shfl(o.x, owner), qy = __shfl(o.y, owner), qz = __shfl(o.z, owner);
        const float ex = __shfl(d.x, owner), ey = __shfl(d.y, owner), ez = __shfl(d.z, owner);
        const float qa = __shfl(a, owner);
        uint32_t hits = 0;
        v2f hb01, cc01, d01, hb23, cc23, d23;
        float4 idf = make_float4(0.f, 0.f, 0.f, 0.f);
        if (act) {
            const float4* g = tg + __umul24(pr & 63u, 5u);
            const float4 q0 = g[0], q1 = g[1], q2 = g[2], q3 = g[3];
            const v2f ox = {qx, qx}, oy = {qy, qy}, oz = {qz, qz};
            const v2f dx = {ex, ex}, dy = {ey, ey}, dz = {ez, ez}, a2 = {qa, qa};
            pair_disc_cc(ox, oy, oz, dx, dy, dz, a2, q0, q1, hb01, cc01, d01);
            pair_disc_cc(ox, oy, oz, dx, dy, dz, a2, q2, q3, hb23, cc23, d23);
            hits = push_sign(0u, hit_sign(hb23.y, cc23.y, d23.y));
            hits = push_sign(hits, hit_sign(hb23.x, cc23.x, d23.x));
            hits = push_sign(hits, hit_sign(hb01.y, cc01.y, d01.y));
            hits = push_sign(hits, hit_sign(hb01.x, cc01.x, d01.x));
            if (hits) idf = g[4];
        }
        // list the candidates (a full list is resolved first)
        uint32_t ctot;
        const uint32_t cpre = wave_prefix((uint32_t)__popc(hits), ctot);
        if (ncand + ctot > (uint32_t)kCandCap) {
            __builtin_amdgcn_wave_barrier();
            resolve_cands(ws, ncand, rank, nact);
            __builtin_amdgcn_wave_barrier();
            ncand = 0;
        }
        const bool direct = ctot > (uint32_t)kCandCap;  // more than the list holds: in place
        uint32_t pos = ncand + cpre;
        const uint32_t ownbits = (uint32_t)owner << 24;
        while (hits) {
            const int s = __builtin_ctz(hits);
            hits &= hits - 1;
            const float hb = s == 0 ? hb01.x : s == 1 ? hb01.y : s == 2 ? hb23.x : hb23.y;
            const float ds = s == 0 ? d01.x : s == 1 ? d01.y : s == 2 ? d23.x : d23.y;
            const float ix = s == 0 ? idf.x : s == 1 ? idf.y : s == 2 ? idf.z : idf.w;
            if (direct) {
                const float t = candidate_t(hb, ds, qa);
                if (t > 0.001f && t < 1e5f)
                    atomicMin(&ws->key[owner], pack_hit(t, (int)__float_as_uint(ix)));
            } else {
                ws->cand[pos++] =
                    make_float4(hb, ds, qa, __uint_as_float(__float_as_uint(ix) | ownbits));
            }
        }
        if (!direct) ncand += ctot;
    }
    __builtin_amdgcn_wave_barrier();
    resolve_cands(ws, ncand, rank, nact);
    __builtin_amdgcn_wave_barrier();
    return true;
}

template <bool kStats, bool kFlat = false>
__device__ __forceinline__ void scan_culled_lane(const TraceParams& p, const float4* tbound,
                                                 const float4* tgroup, const f3 o, const f3 d,
                                                 float& max_t, int& best,
                                                 uint64_t& groups_tested,
                                                 uint64_t& bounds_tested, uint32_t& lane_cnt,
                                                 uint32_t& rounds, WaveScratch* ws = nullptr) {
    const float a = dot(d, d);
    const float inv = __builtin_amdgcn_rsqf(a);
    CullRay r;
    r.ox = (v2f){o.x, o.x};
    r.oy = (v2f){o.y, o.y};
    r.oz = (v2f){o.z, o.z};
    r.wx = (v2f){d.x * inv, d.x * inv};
    r.wy = (v2f){d.y * inv, d.y * inv};
    r.wz = (v2f){d.z * inv, d.z * inv};
    const v2f dx = {d.x, d.x}, dy = {d.y, d.y}, dz = {d.z, d.z}, a2 = {a, a};
    cfloat4* node = (cfloat4*)p.cnode;
    cfloat4* top = (cfloat4*)p.ctop;
    const int ncg = p.ncgroups;
    for (int gb = 0; gb < p.nbig; ++gb)  // the big spheres, for every ray (scalar loads)
        exact_group_uniform((cfloat4*)p.cgroup + 5 * gb, r, dx, dy, dz, a2, a, max_t, best);
    // per-segment pass counters, wave-uniform: kept in SGPRs, folded into the 64-bit totals once
    uint32_t n_bounds = 0, n_groups = (uint32_t)p.nbig;
    const uint32_t lane = threadIdx.x & 63u;
    if constexpr (kFlat) ws->key[lane] = pack_hit(max_t, best);
    uint32_t tops = 0;
    for (int base = 0; base < ncg; base += 64) {
        // level 0, wave-uniform: the chunk's own bound (two chunks per test), per-lane bits
        if ((base & 127) == 0) {
            const BoundPair tp = load_bound_pair(top + 3 * (base >> 7));
            tops = ~push_bound_pair(0u, r, tp.b0, tp.b1, tp.b2) & 3u;
            n_bounds += 2;
        }
        const bool in_chunk = ((tops >> ((base >> 6) & 1)) & 1u) != 0;
        if (__ballot(in_chunk) == 0) continue;
        // level 1, wave-uniform: nodes of this chunk, per-lane bits
        const int nn = min(8, (ncg - base) >> 3);
        cfloat4* nb = node + 3 * (base >> 4);
        // sign bits pushed from the last node down, so bit j ends up = node j ruled out
        uint32_t out = 0;
        BoundPair cur = load_bound_pair(nb + 3 * ((nn - 2) >> 1));
        for (int j = nn - 2; j >= 0; j -= 2) {
            const BoundPair nxt = load_bound_pair(nb + 3 * ((j >= 2 ? j - 2 : j) >> 1));
            out = push_bound_pair(out, r, cur.b0, cur.b1, cur.b2);
            cur = nxt;
        }
        uint32_t nodes = in_chunk ? ~out & ((1u << nn) - 1u) : 0u;
        n_bounds += (uint32_t)nn;
        // level 2, per lane: the groups of this lane's nodes
        uint64_t need = 0;
        while (__ballot(nodes != 0)) {
            n_bounds += 8;  // one wave pass = 8 bound tests
            if (nodes) {
                const int j = __builtin_ctz(nodes);
                nodes &= nodes - 1;
                const float4* gb = tbound + 3 * (base >> 1) + __umul24((uint32_t)j, 12u);
                uint32_t gout = 0;
#pragma unroll
                for (int k = 3; k >= 0; k--) {
                    const float4 b0 = gb[3 * k], b1 = gb[3 * k + 1], b2 = gb[3 * k + 2];
                    gout = push_bound_pair(gout, r, b0, b1, make_float2(b2.x, b2.y));
                }
                need |= (uint64_t)(~gout & 0xffu) << (8 * j);
            }
        }
        if constexpr (kStats) lane_cnt += (uint32_t)__popcll(need);
        if constexpr (kFlat) {
            if (exact_flat(ws, tgroup + 5 * base, need, o, d, a, lane, n_groups)) continue;
            // too many pairs for the list: the per-lane loop, on registers synced with the key
            __builtin_amdgcn_wave_barrier();
            const unsigned long long k = ws->key[lane];
            max_t = __uint_as_float((uint32_t)(k >> 32));
            best = (int)(uint32_t)k;
        }
        // the exact test, per lane on its own groups
        while (__ballot(need != 0)) {
            ++n_groups;
            uint32_t cand = 0;  // stats: candidate roots this lane evaluates in this pass
            if (need) {
                const int k = __builtin_ctzll(need);
                need &= need - 1;
                const float4* g = tgroup + 5 * base + __umul24((uint32_t)k, 5u);
                const float4 q0 = g[0], q1 = g[1], q2 = g[2], q3 = g[3], idf = g[4];
                v2f hb01, cc01, d01, hb23, cc23, d23;
                pair_disc_cc(r.ox, r.oy, r.oz, dx, dy, dz, a2, q0, q1, hb01, cc01, d01);
                pair_disc_cc(r.ox, r.oy, r.oz, dx, dy, dz, a2, q2, q3, hb23, cc23, d23);
                const int i0 = __float_as_int(idf.x), i1 = __float_as_int(idf.y),
                          i2 = __float_as_int(idf.z), i3 = __float_as_int(idf.w);
                // bit s = member s may be accepted (sign bits, pushed from member 3 down)
                uint32_t hits = push_sign(0u, hit_sign(hb23.y, cc23.y, d23.y));
                hits = push_sign(hits, hit_sign(hb23.x, cc23.x, d23.x));
                hits = push_sign(hits, hit_sign(hb01.y, cc01.y, d01.y));
                hits = push_sign(hits, hit_sign(hb01.x, cc01.x, d01.x));
                if constexpr (kStats) cand = __popc(hits);
                while (hits) {
                    const int s = __builtin_ctz(hits);
                    hits &= hits - 1;
                    const float hb = s == 0 ? hb01.x : s == 1 ? hb01.y : s == 2 ? hb23.x : hb23.y;
                    const float ds = s == 0 ? d01.x : s == 1 ? d01.y : s == 2 ? d23.x : d23.y;
                    const int idx = s == 0 ? i0 : s == 1 ? i1 : s == 2 ? i2 : i3;
                    consider(candidate_t(hb, ds, a), idx, max_t, best);
                }
            }
            if constexpr (kStats) {  // wave passes of the candidate loop = max over lanes
                for (int off = 32; off > 0; off >>= 1)
                    cand = max(cand, (uint32_t)__shfl_xor((int)cand, off));
                rounds += cand;
            }
        }
        if constexpr (kFlat) ws->key[lane] = pack_hit(max_t, best);
    }
    if constexpr (kFlat) {
        __builtin_amdgcn_wave_barrier();
        const unsigned long long k = ws->key[lane];
        max_t = __uint_as_float((uint32_t)(k >> 32));
        best = (int)(uint32_t)k;
    }
    bounds_tested += __builtin_amdgcn_readfirstlane(n_bounds);
    groups_tested += __builtin_amdgcn_readfirstlane(n_groups);
}

// Local element q = 64 * lt + slot of this rank -> pixel (x, y) and its framebuffer index.
struct Pixel {
    uint32_t x, y, out_index;
    bool valid;  // edge tiles of frames that are not multiples of 8 are partial
};

__device__ __forceinline__ Pixel pixel_of(uint32_t q, uint32_t W, uint32_t H, uint32_t tiles_x,
                                          uint32_t world, uint32_t rank) {
    const uint32_t lt = q >> 6, slot = q & 63u;
    uint32_t tx, ty;
    tile_of(lt, rank, world, tiles_x, &tx, &ty);
    Pixel px;
    px.x = 8u * tx + (slot & 7u);
    px.y = 8u * ty + (slot >> 3);
    px.valid = px.x < W && px.y < H;
    px.out_index = world == 1u ? px.y * W + px.x : q;
    return px;
}

// kCull: 0 = linear scan (kLds: table in LDS), 1 = culled scan, 2 = per-lane culled scan
// with the group tables copied to LDS, 3 = per-lane culled scan on global tables.
template <bool kLds, bool kStats, int kCull = 0>
__device__ __forceinline__ void trace_impl(const TraceParams& p, float4* lds_geom) {
    const int n = p.nspheres;
    if constexpr (kLds) {
        const int nq = 4 * (((n + 3) >> 2) + 1);
        for (int i = threadIdx.x; i < nq; i += blockDim.x) lds_geom[i] = p.geom[i];
        __syncthreads();
    }
    const float4* tbound = p.cbound;
    const float4* tgroup = p.cgroup + 5 * p.nbig;  // the hierarchy's group records
    WaveScratch* ws = nullptr;
    if constexpr (kCull == 2 || kCull == 4) {
        const int nb = (p.ncgroups >> 1) * 3, ng = p.ncgroups * 5;
        for (int i = threadIdx.x; i < nb; i += blockDim.x) lds_geom[i] = p.cbound[i];
        for (int i = threadIdx.x; i < ng; i += blockDim.x) lds_geom[nb + i] = tgroup[i];
        __syncthreads();
        tbound = lds_geom;
        tgroup = lds_geom + nb;
        if constexpr (kCull == 4)
            ws = reinterpret_cast<WaveScratch*>(lds_geom + nb + ng) + (threadIdx.x >> 6);
    }
    const uint32_t lane = threadIdx.x & 63u;
    const f3 p00 = mk(p.cam[0], p.cam[1], p.cam[2]);
    const f3 du = mk(p.cam[3], p.cam[4], p.cam[5]);
    const f3 dv = mk(p.cam[6], p.cam[7], p.cam[8]);
    const f3 cam = mk(p.cam[9], p.cam[10], p.cam[11]);
    const float spp_f = (float)p.spp;
    const uint32_t nchunks = (uint32_t)p.nchunks;
    const bool reverse = (p.flags & kFlagReverseOrder) != 0;

    bool done = false, need = true;
    int sample = 0, sample_end = 0, pass = 0;
    uint32_t q = 0, chunk = 0, out_index = 0;
    f3 pc = mk(0.f, 0.f, 0.f), o = pc, d = pc, atten = pc, acc = pc;
    unsigned long long segs = 0;
    uint64_t st_iters = 0, st_active = 0, st_hitgroups = 0, st_fetch = 0;
    uint64_t w_groups = 0, w_bounds = 0;  // per wave (uniform): sphere groups / bounds tested
    // the wave's current block of items (wave-uniform); 64 = exhausted, fetch a new one
    const uint32_t total_blocks = p.total_items >> 6;
    uint32_t blk_next = 64u, blk_lt = 0u, blk_chunk = 0u, blk_tx = 0u, blk_ty = 0u;

    for (;;) {
        // ---- lanes whose item is finished take the next slots of the wave's current block
        //      (one tile x chunk = 64 items); a new block costs one atomic per wave ----
        uint64_t need_mask = __ballot(need && !done);
        while (need_mask) {
            if (blk_next >= 64u) {
                if constexpr (kStats && kCull == 0) ++st_fetch;
                const int leader = __ffsll((unsigned long long)__ballot(1)) - 1;
                uint32_t b = 0;
                if ((int)lane == leader) b = atomicAdd(p.work, 1u);
                b = __builtin_amdgcn_readfirstlane(__shfl(b, leader));
                if (b >= total_blocks) {  // queue drained: lanes still wanting work are done
                    if (need) done = true;
                    break;
                }
                if (reverse) b = total_blocks - 1u - b;
                // block b = (local tile lt, chunk): wave-uniform tile origin and sample range
                blk_lt = b / nchunks;
                blk_chunk = b - blk_lt * nchunks;
                tile_of(blk_lt, (uint32_t)p.rank, (uint32_t)p.world, p.tiles_x, &blk_tx, &blk_ty);
                blk_next = 0u;
            }
            const uint32_t avail = 64u - blk_next;
            const uint32_t mine = lanes_below(need_mask);
            if (need && !done && mine < avail) {
                const uint32_t slot = blk_next + mine;
                const uint32_t px = 8u * blk_tx + (slot & 7u), py = 8u * blk_ty + (slot >> 3);
                if (px < (uint32_t)p.width && py < (uint32_t)p.height) {  // edge tiles: skip
                    chunk = blk_chunk;
                    q = blk_lt * 64u + slot;
                    out_index = p.world == 1 ? py * (uint32_t)p.width + px : q;
                    // shader.comp:43  pixel00 + x*delta_u + y*delta_v
                    pc = add(add(p00, scale((float)px, du)), scale((float)py, dv));
                    acc = mk(0.f, 0.f, 0.f);
                    sample = (int)(chunk * (uint32_t)p.chunk);
                    sample_end = min(sample + p.chunk, p.spp);
                    // first camera ray of the chunk, shader.comp:48-52
                    const float2 jt = p.jitter[sample];
                    const f3 ps = add(pc, add(scale(jt.x, du), scale(jt.y, dv)));
                    o = cam;
                    d = sub(ps, cam);
                    atten = mk(1.f, 1.f, 1.f);
                    pass = 0;
                    need = false;
                }
            }
            blk_next += min((uint32_t)__popcll(need_mask), avail);
            need_mask = __ballot(need && !done);
        }
        const uint64_t live = __ballot(!done);
        if (live == 0) break;
        if constexpr (kStats) {
            ++st_iters;
            st_active += (uint64_t)__popcll(live);
        }
        if (done) continue;

        // ---- one segment: scan the whole sphere list (functions.glsl:73-81) ----
        ++segs;
        float max_t = 1e5f;
        int best = -1;
        uint32_t hit_groups = 0;
        if constexpr (kCull != 0) {
            // culling needs every ray of the wave in the guarded finite range (see above)
            const float aa = dot(d, d);
            const bool guarded = (p.flags & kFlagSceneBounded) != 0 && aa >= 0x1p-20f &&
                                 aa <= 0x1p60f && fabsf(o.x) <= 0x1p30f &&
                                 fabsf(o.y) <= 0x1p30f && fabsf(o.z) <= 0x1p30f;
            if (__ballot(!guarded) == 0) {
                uint32_t lane_cnt = 0;
                if constexpr (kCull == 1)
                    scan_culled<kStats>(p, o, d, max_t, best, w_groups, w_bounds, hit_groups,
                                        lane_cnt);
                else if constexpr (kCull == 4)
                    scan_culled_lane<kStats, true>(p, tbound, tgroup, o, d, max_t, best,
                                                   w_groups, w_bounds, lane_cnt, hit_groups, ws);
                else
                    scan_culled_lane<kStats>(p, tbound, tgroup, o, d, max_t, best, w_groups,
                                             w_bounds, lane_cnt, hit_groups);
                if constexpr (kStats) {  // CULL stats: debug[3] = sum of per-wave max lane need
                    for (int off = 32; off > 0; off >>= 1)
                        lane_cnt = max(lane_cnt, (uint32_t)__shfl_xor((int)lane_cnt, off));
                    st_fetch += lane_cnt;
                }
            } else {
                scan_spheres<false>(p, lds_geom, n, o, d, max_t, best, hit_groups);
                w_groups += (uint64_t)((n + 3) >> 2);
            }
        } else {
            scan_spheres<kLds>(p, lds_geom, n, o, d, max_t, best, hit_groups);
            w_groups += (uint64_t)((n + 3) >> 2);
        }
        if constexpr (kStats) st_hitgroups += hit_groups;

        // ---- shade (textures.glsl) or sky (functions.glsl:85-89) ----
        bool ended = false;
        f3 contrib = mk(0.f, 0.f, 0.f);
        if (best >= 0) {
            const float4 cr = p.center_radius[best];
            const float4 sh = p.shade[best];
            const float mat = p.material[best];
            const f3 point = add(scale(max_t, d), o);
            const f3 normal = divs(sub(point, mk(cr.x, cr.y, cr.z)), cr.w);
            const int type = (int)mat;
            const f3 albedo = mk(sh.x, sh.y, sh.z);
            const float param = sh.w;
            // first rand: rand(dir.xy) for lambertian/metal, rand(point.xy) for glass
            const float r1 = (type == 3) ? rand2(point.x, point.y) : rand2(d.x, d.y);
            if (type == 1 || type == 2) {
                const float r2 = rand2(d.x, d.z);
                const float r3 = rand2(d.y, d.z);
                const f3 u = normalize(mk(r1, r2, r3));  // random_in_unit_sphere(dir)
                if (type == 1) {
                    d = add(normal, u);
                    atten = scale(param, mul(atten, albedo));
                } else {
                    d = add(reflect(d, normal), scale(param, u));
                    atten = mul(atten, albedo);
                }
                o = point;
            } else if (type == 3) {
                const f3 reflected = reflect(d, normal);
                f3 outward;
                float ni, cosine;
                const float dn = dot(d, normal);
                if (dn > 0.0f) {
                    outward = neg(normal);
                    ni = param;
                    cosine = __builtin_sqrtf(1.0f - param * param * (1.0f - dn * dn));
                } else {
                    outward = normal;
                    ni = 1.0f / param;
                    cosine = -dn;
                }
                f3 refracted = mk(0.f, 0.f, 0.f);
                float reflect_prob = 1.0f;
                const float dt = dot(d, outward);
                const float disc = 1.0f - ni * ni * (1.0f - dt * dt);
                if (disc > 0.0f) {
                    const float sd = __builtin_sqrtf(disc);
                    refracted = sub(scale(ni, sub(d, scale(dt, outward))), scale(sd, outward));
                    reflect_prob = schlick(cosine, param);
                }
                o = point;
                d = (r1 < reflect_prob) ? reflected : refracted;
            }
            ++pass;
            if (pass >= p.max_depth) ended = true;  // undefined GLSL return -> vec3(0)
        } else {
            const float len = length(d);
            const float t = 0.5f * (d.y / len + 1.0f);
            const float om = 1.0f - t;
            contrib = mul(atten, mk(om + 0.5f * t, om + 0.7f * t, om + t));
            ended = true;
        }

        if (ended) {
            acc = add(acc, contrib);
            ++sample;
            if (sample == sample_end) {
                if ((p.flags & kFlagSlab) == 0u)
                    p.out[out_index] =
                        make_float4(acc.x / spp_f, acc.y / spp_f, acc.z / spp_f, 1.0f);
                else
                    p.partial[(size_t)chunk * (p.local_tiles * 64u) + q] =
                        make_float4(acc.x, acc.y, acc.z, 0.0f);
                need = true;
            } else {
                const float2 jt = p.jitter[sample];
                const f3 ps = add(pc, add(scale(jt.x, du), scale(jt.y, dv)));
                o = cam;
                d = sub(ps, cam);
                atten = mk(1.f, 1.f, 1.f);
                pass = 0;
            }
        }
    }

    // one segment-counter atomic per wave
    unsigned long long total = segs;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) total += __shfl_xor(total, off);
    if (lane == 0 && total) atomicAdd(p.segments, total);
    if (lane == 0 && p.work_done) {
        atomicAdd(p.work_done + 0, (unsigned long long)w_groups);
        atomicAdd(p.work_done + 1, (unsigned long long)w_bounds);
    }
    if constexpr (kStats) {
        if (lane == 0 && p.debug) {
            atomicAdd(p.debug + 0, (unsigned long long)st_iters);
            atomicAdd(p.debug + 1, (unsigned long long)st_active);
            atomicAdd(p.debug + 2, (unsigned long long)st_hitgroups);
            atomicAdd(p.debug + 3, (unsigned long long)st_fetch);
            const unsigned long long t = __builtin_amdgcn_s_memrealtime();
            atomicMax(p.debug + 4, t);
            atomicMin(p.debug + 5, t);
            atomicAdd(p.debug + 6, t >> 8);  // mean wave end time (in 256-tick units)
            atomicAdd(p.debug + 7, 1ull);
        }
    }
}

}  // namespace

extern "C" __global__ __launch_bounds__(256) void vcrt_trace_lds(TraceParams p) {
    extern __shared__ __attribute__((aligned(16))) float4 lds_geom[];
    trace_impl<true, false>(p, lds_geom);
}

extern "C" __global__ __launch_bounds__(256) void vcrt_trace_smem(TraceParams p) {
    trace_impl<false, false>(p, nullptr);
}

// Culled scan (exact; see scan_culled): spatially grouped sphere table + wave-level group tests.
extern "C" __global__ __launch_bounds__(256) void vcrt_trace_cull(TraceParams p) {
    trace_impl<false, false, 1>(p, nullptr);
}

extern "C" __global__ __launch_bounds__(256) void vcrt_trace_cull_stats(TraceParams p) {
    trace_impl<false, true, 1>(p, nullptr);
}

// Per-lane culled scan (scan_culled_lane): tables in LDS (dynamic size = group-pair bounds +
// group records) or read from global memory.
extern "C" __global__ __launch_bounds__(256) void vcrt_trace_cull_lane_lds(TraceParams p) {
    extern __shared__ __attribute__((aligned(16))) float4 lds_tab[];
    trace_impl<false, false, 2>(p, lds_tab);
}

extern "C" __global__ __launch_bounds__(256) void vcrt_trace_cull_lane_lds_stats(TraceParams p) {
    extern __shared__ __attribute__((aligned(16))) float4 lds_tab[];
    trace_impl<false, true, 2>(p, lds_tab);
}

// Per-lane scan with the exact phase flattened over the wave (exact_flat): LDS tables plus
// 3.5 KB of scratch per wave.
extern "C" __global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(5))) void vcrt_trace_cull_flat(TraceParams p) {
    extern __shared__ __attribute__((aligned(16))) float4 lds_tab[];
    trace_impl<false, false, 4>(p, lds_tab);
}

extern "C" __global__ __launch_bounds__(256) void vcrt_trace_cull_flat_stats(TraceParams p) {
    extern __shared__ __attribute__((aligned(16))) float4 lds_tab[];
    trace_impl<false, true, 4>(p, lds_tab);
}

// The same with 1024-thread workgroups: one table copy serves 16 waves, so tables of up to
// 160 KB (the whole LDS of a CU; 4100 spheres take 108 KB) still live in LDS.
extern "C" __global__ __launch_bounds__(1024) void vcrt_trace_cull_lane_lds_wide(TraceParams p) {
    extern __shared__ __attribute__((aligned(16))) float4 lds_tab[];
    trace_impl<false, false, 2>(p, lds_tab);
}

extern "C" __global__ __launch_bounds__(1024) void vcrt_trace_cull_lane_lds_wide_stats(
    TraceParams p) {
    extern __shared__ __attribute__((aligned(16))) float4 lds_tab[];
    trace_impl<false, true, 2>(p, lds_tab);
}

extern "C" __global__ __launch_bounds__(256) void vcrt_trace_cull_lane(TraceParams p) {
    trace_impl<false, false, 3>(p, nullptr);
}

extern "C" __global__ __launch_bounds__(256) void vcrt_trace_cull_lane_stats(TraceParams p) {
    trace_impl<false, true, 3>(p, nullptr);
}

// Diagnostics builds (VCRT_DEBUG_STATS=1): same kernels plus lane-occupancy/tail counters.
extern "C" __global__ __launch_bounds__(256) void vcrt_trace_lds_stats(TraceParams p) {
    extern __shared__ __attribute__((aligned(16))) float4 lds_geom[];
    trace_impl<true, true>(p, lds_geom);
}

extern "C" __global__ __launch_bounds__(256) void vcrt_trace_smem_stats(TraceParams p) {
    trace_impl<false, true>(p, nullptr);
}

// Chunk sums -> pixels in chunk order: ((P0 + P1) + P2) + ..., then / spp (shader.comp:56).
extern "C" __global__ __launch_bounds__(256) void vcrt_resolve(ResolveParams p) {
    const uint32_t elems = p.local_tiles * 64u;
    for (uint32_t q = blockIdx.x * blockDim.x + threadIdx.x; q < elems;
         q += gridDim.x * blockDim.x) {
        const Pixel px = pixel_of(q, (uint32_t)p.width, (uint32_t)p.height, p.tiles_x,
                                  (uint32_t)p.world, (uint32_t)p.rank);
        if (!px.valid) continue;
        float4 s = p.accum ? p.accum[q] : make_float4(0.f, 0.f, 0.f, 0.f);
        for (int c = 0; c < p.nchunks; ++c) {  // 0 + P0 == P0: the first chunk is exact
            const float4 v = p.partial[(size_t)c * elems + q];
            s.x = s.x + v.x;
            s.y = s.y + v.y;
            s.z = s.z + v.z;
        }
        if (p.accum) p.accum[q] = s;
        p.out[px.out_index] =
            make_float4(s.x / p.spp_total, s.y / p.spp_total, s.z / p.spp_total, 1.0f);
    }
}

// Re-interleave the packed tile framebuffers gathered from every rank into one frame.
extern "C" __global__ __launch_bounds__(256) void vcrt_assemble(AssembleParams p) {
    const uint32_t W = (uint32_t)p.width;
    const uint32_t total = W * (uint32_t)p.height;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < total;
         i += gridDim.x * blockDim.x) {
        const uint32_t y = i / W, x = i - y * W;
        uint32_t r, lt;
        owner_of(x >> 3, y >> 3, (uint32_t)p.world, p.tiles_x, &r, &lt);
        const uint32_t slot = ((y & 7u) << 3) | (x & 7u);
        p.frame[i] = p.gathered[((size_t)r * p.tiles_per_rank + lt) * 64u + slot];
    }
}

// sRGB8 encode (present-time conversion of the B8G8R8A8_SRGB swapchain, Frontend.cpp:43):
// a channel's byte is the number of the 255 host-computed thresholds it reaches, i.e. the
// round-to-nearest of the exact sRGB encode of the clamped value; alpha is stored linearly.
extern "C" __global__ __launch_bounds__(256) void vcrt_encode_srgb8(EncodeParams p) {
    __shared__ float th[256];
    for (int i = threadIdx.x; i < 256; i += blockDim.x) th[i] = i < 255 ? p.thresholds[i] : 3e38f;
    __syncthreads();
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < p.count;
         i += gridDim.x * blockDim.x) {
        const float4 v = p.in[i];
        const float c[3] = {v.x, v.y, v.z};
        unsigned char b[3];
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            int lo = 0;  // count of thresholds <= c[k] (NaN reaches none: 0)
#pragma unroll
            for (int step = 128; step > 0; step >>= 1)
                if (c[k] >= th[lo + step - 1]) lo += step;
            b[k] = (unsigned char)lo;
        }
        const float a = v.w != v.w ? 0.0f : fminf(fmaxf(v.w, 0.0f), 1.0f);
        p.out[i] = make_uchar4(b[0], b[1], b[2], (unsigned char)(a * 255.0f + 0.5f));
    }
}

extern "C" __global__ __launch_bounds__(256) void vcrt_fill(FillParams p) {
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < p.count;
         i += gridDim.x * blockDim.x)
        p.out[i] = p.value;
}
