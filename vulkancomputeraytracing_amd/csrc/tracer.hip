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
//   * Work items are (pixel, chunk of K samples): a block of 64 items holds all the chunks of a
//     few pixels of one 8x8 tile (chunk-minor), and a wave takes a whole block with one atomic on
//     its XCD's work queue and hands its items to lanes as they free up; a lane whose path ends
//     starts its next sample at once (path regeneration). A lane sums its samples in fp32 in
//     quanta of G (vcrt_math.h "Accumulation"); each quantum sum, quantized by the scene's scale
//     2^s, is added exactly to the pixel's sums (LDS atomics into the wave's accumulation ring,
//     flushed to global memory per pixel) and vcrt_resolve divides: the image depends on G and s
//     only, not on the work items, the schedule or the number of GPUs. One quantum per pixel:
//     the lane writes the pixel.
//   * Ray state lives in VGPRs. Sphere tests run two spheres per packed-fp32 instruction
//     (v_pk_add_f32 / v_pk_mul_f32 on pair-SoA groups of four: 2 lane-ops per issue, the only
//     way gfx950 reaches its fp32 peak).
//   * The sphere-list scan is either the reference's linear scan (wave-uniform groups through
//     the scalar cache or LDS) or an exact culled scan over a spatial hierarchy (groups of 4,
//     nodes of 8 groups, chunks of 64 groups), wave-uniform or per lane on an LDS copy of the
//     tables; see "Culled scan" below for why it returns the same sphere and t. In the flat
//     culled scan a camera ray starts from its pixel quarter's precomputed group list
//     (csrc/primary.cpp) instead of the hierarchy.
//   * Only fp32 add/sub/mul plus correctly rounded div/sqrt, no contraction, in everything
//     that reaches the image: results are bit-identical to the CPU oracle for the same
//     accumulation order. No MFMA.
#include <hip/hip_runtime.h>

#include <type_traits>

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

// Issued-work tallies (TraceParams.work_done): a wave-uniform count x is credited to the wave's
// first active lane, so the sum over the lanes is the wave's total. (A per-wave 64-bit counter
// is per lane under SIMT all the same -- lanes that skip a region keep their old value -- and
// lived in VGPR pairs that spilled, with a full vmcnt wait at every update.)
__device__ __forceinline__ void tally(uint32_t& t, uint32_t x) {
    const uint32_t first = (uint32_t)__builtin_ctzll(__builtin_amdgcn_read_exec());
    t += (threadIdx.x & 63u) == first ? x : 0u;
}

// tally into a per-wave LDS counter (the flat scans' WaveScratch::work): one LDS add from the
// first active lane, nothing held in VGPRs across the loop
__device__ __forceinline__ void tally_lds(uint32_t* slot, uint32_t x) {
    const uint32_t first = (uint32_t)__builtin_ctzll(__builtin_amdgcn_read_exec());
    if ((threadIdx.x & 63u) == first) atomicAdd(slot, x);
}

// Region counters of the stats builds (tools/valu_attrib.py): one global atomic by the wave's
// first active lane into the wave's own row of TraceParams.region ([waves][kRegions]) each time
// the wave enters a counted region with some lane active. The product kernels pass a null row,
// which folds every call away.
namespace reg {
enum : uint32_t {
    kIter = 0, kRetire, kRetireNan, kRetireRing, kRetireGlobal, kNewRay, kFetchTrip, kBlock,
    kBlockRing, kItem, kCam, kCamBig, kCamBigM0, kCamBigM1, kCamBigM2, kCamBigM3, kCamListTrip,
    kCamRootTrip, kShadeCam, kScan, kScanLinear, kMainBig, kMainBigM0, kMainBigM1, kMainBigM2,
    kMainBigM3, kListed, kLevelChunk, kLevelNodes, kDrainTrip, kPassCand, kPassGroup, kPassNode,
    kPassChunk, kShadeSkyMain, kSqrtFallback, kDivFallback, kSteal,
    kShadeBase0 = 40, kShadeBase1 = 56,  // the shading's regions, per call site (camera phase,
                                         // main-scan sky), at these offsets:
    kShEntry = 0, kShHit, kShNormalDiv, kShSinFallback, kShLamMetal, kShLam, kShMetal, kShGlass,
    kShGlassIn, kShGlassOut, kShGlassRefract, kShSky, kShEnded, kShNewRay, kShItemEnd,
    // sub-blocks of the flat scan's regions that run only on some of their entries
    kPrefixSlow = 72, kLevelTop, kPushNode, kPushGroup, kPushLevel, kListedTrip,
    kCount = 88
};
}  // namespace reg
constexpr uint32_t kRegions = 88;  // the host's row size (vcrt_kernel_abi.h TraceParams.region)

__device__ __forceinline__ void region(uint32_t* row, uint32_t k) {
    if (row) {
        const uint32_t first = (uint32_t)__builtin_ctzll(__builtin_amdgcn_read_exec());
        if ((threadIdx.x & 63u) == first) atomicAdd(row + k, 1u);
    }
}

typedef __attribute__((address_space(4))) const float4 cfloat4;

// A 32-bit constant materialized in a VGPR where it is used: the asm is volatile, so it is not
// hoisted out of the persistent loop. Left to itself the compiler keeps constant pairs such as a
// scan's initial (max_t, best) = (kInfinity, -1) live across the loop, and under the flat
// kernel's register pressure spills them to scratch: a scratch load and a vmcnt wait per use.
static_assert(__builtin_bit_cast(uint32_t, kInfinity) == 0x47c35000u, "vconst<kInfinity bits>");
template <uint32_t kC>
__device__ __forceinline__ uint32_t vconst() {
    uint32_t r;
    asm volatile("v_mov_b32 %0, %1" : "=v"(r) : "i"(kC));
    return r;
}

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
    const float min_t = kMinT;
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
    const float min_t = kMinT;
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
//      box's members (radius >= r_b, all |c| <= c_max, r <= r_max) M_s <= M_b = K_b Q with
//      K_b = 8.1u / r_b and Q = (|o| + c_max)^2 + r_max^2.
//  (3) the box test. Group, node and chunk bounds are axis-aligned boxes B = [lo, hi] of their
//      members (rounded outwards) with their K_b. Per axis the lane computes the plane
//      parameters fma(lo, inv, c), fma(hi, inv, c) with inv = v_rcp(d') (1 ulp), c = -o inv,
//      d' = d with components below 2^-40 raised to 2^-40; tnear = max of the per-axis minima,
//      tfar = min of the maxima, and rules B out when
//        gap = fma(K_b, c2, (tfar - tnear) + c1) < 0,
//        c1 = 1.001 J 5.1u (L + |o|_inf),  c2 = 1.001 J Q,  J = 2 max_i |inv_i|,
//      L = max |box coordinate|. Why: if the real line met B grown by M_b at t*, every exact
//      per-axis interval of B would reach within (M_b + dc) / |d'_i| of t*, where dc <=
//      sqrt(3) 2^-30 (L + M_b + |o|_inf) bounds the shift from d to d' (a >= 2^-20); each
//      computed end lies within 4.02u (L + |o_i|) / |d'_i| of its exact value (rcp 2u, two
//      roundings); and 1 / |d'_i| <= (1 + 2.01u) J / 2. So tfar - tnear >= -(M_b + dc + 4.02u
//      (L + |o|_inf)) (1 + 2.01u) J, which c1 + K_b c2 exceeds by more than the last three
//      roundings: gap >= 0, the box is kept. Hence a ruled-out box holds no member with
//      disc_f >= 0. (Q and the 1.001 factors absorb the per-ray roundings; K_b = inf, a zero
//      radius, keeps its box.) The host passes K_b, c_max, r_max^2 and L rounded up.
//  (4) behind the origin. A member is accepted only if hb_f < 0 or cc_f < 0 (may_hit). If the
//      line meets the member's sphere grown by M_s only at t < -tau (or not at all), with
//      tau^2 = 5.02u Q / a, then exactly hb = -a t_c > a tau >= 4.02u |oc| |d| (t_c: the
//      centre's parameter) and cc = |oc|^2 - r^2 > a tau^2 >= 5.02u (|oc|^2 + r^2), which
//      the roundings of hb_f (4.02u |oc| |d|: oc and the dot) and of cc_f (5.02u |oc|^2 and u r^2)
//      cannot flip: hb_f >= 0 and cc_f >= 0, rejected. So an accepted member's grown sphere,
//      inside the grown box, meets the line at some t* >= -tau, and the computed far end is at
//      least t* - (c1 + K_b c2) / 2 by (3). The kernels shift every plane by tau (c = fma(-o,
//      inv, tau): t' = t + tau, gaps unchanged; the shift's roundings, below 4.1u tau, fit in
//      c1's spare) and clamp the near end at 0: gap = fma(K_b, c2, (tf' - max(tn', 0)) + c1)
//      rules a box out when its whole stretch of the line lies behind -tau as well.
//      (tau = sqrt(3.2e-7 Q / a), 7% above 5.02u Q / a for the roundings of Q, 1/a and sqrt.)
// Waves holding a ray outside the guarded range scan the original table in reference order.

// t of one candidate as hit_sphere would accept it (finite case, fact (1)).
__device__ __forceinline__ float candidate_t(float hb, float disc, float a) {
    const float sq = __builtin_sqrtf(disc);
    const float r1 = (-hb - sq) / a;
    if (r1 > kMinT) return r1;
    return (-hb + sq) / a;
}

// candidate_t for a ray of the guarded range (a in [2^-20, 2^60], |o|, |c|, r <= 2^30, so
// |hb| < 2^63 and disc < 2^126), with ya = recip_a(a) computed once per ray. It returns the
// same t as candidate_t wherever that t can be accepted, and a t <= min_t wherever candidate_t's
// is (the only other use of a root: candidate_t's choice between them):
//  * division: hipcc's correctly rounded x / a is v_div_scale (x2), a Newton-refined v_rcp,
//    q0 = x y, two residual corrections (the second in v_div_fmas) and v_div_fixup. v_div_scale
//    leaves both operands alone and v_div_fmas does not rescale when x, a are normal, x / a is
//    normal and exp(x) - exp(a) < 96, exp(x) > 23 (the ISA's V_DIV_SCALE_F32); v_div_fixup only
//    changes special values. div_a runs that unscaled sequence: for |x| in [2^-103, 2^64) the
//    same bits. A root that can be accepted (> min_t = 0.001 with a >= 2^-20) has |x| > 2^-30.
//    For |x| < 2^-103 (or x = 0) both quotients are below 2^-83 in magnitude, so both roots
//    are rejected alike (their sign or last bits never matter).
//  * sqrt: hipcc's correctly rounded sqrt scales x < 2^-96, takes v_sqrt and picks between its
//    neighbours by two FMA residuals, then special-cases 0 and inf; sqrt_unscaled runs the
//    unscaled middle, the same bits for x in [2^-96, 2^126]. Lanes with disc < 2^-96 take the
//    full sqrt (a zero discriminant, a grazing ray).
__device__ __forceinline__ float recip_a(float a) {
    const float y0 = __builtin_amdgcn_rcpf(a);
    return __builtin_fmaf(__builtin_fmaf(-a, y0, 1.0f), y0, y0);
}

__device__ __forceinline__ float div_a(float x, float a, float ya) {
    const float q0 = x * ya;
    const float q1 = __builtin_fmaf(__builtin_fmaf(-a, q0, x), ya, q0);
    return __builtin_fmaf(__builtin_fmaf(-a, q1, x), ya, q1);
}

__device__ __forceinline__ float sqrt_unscaled(float x) {
    const float s = __builtin_amdgcn_sqrtf(x);
    const float sm = __uint_as_float(__float_as_uint(s) - 1u);
    const float sp = __uint_as_float(__float_as_uint(s) + 1u);
    float r = __builtin_fmaf(-sm, s, x) <= 0.0f ? sm : s;
    return __builtin_fmaf(-sp, s, x) > 0.0f ? sp : r;
}

// Correctly rounded sqrt for any x: the unscaled sequence, and hipcc's full one in a real branch
// for lanes outside [2^-96, inf] (tiny, zero, negative or NaN x).
__device__ __forceinline__ float sqrt_fast(float x, uint32_t* rrow = nullptr) {
    float r = sqrt_unscaled(x);
    if (__ballot(!(x >= 0x1p-96f))) {  // wave-uniform: no exec-mask save and restore
        asm volatile("");
        region(rrow, reg::kSqrtFallback);
        const float full = __builtin_sqrtf(x);
        r = !(x >= 0x1p-96f) ? full : r;
    }
    return r;
}

__device__ __forceinline__ float candidate_t_fast(float hb, float disc, float a, float ya,
                                                  uint32_t* rrow = nullptr) {
    float sq = sqrt_unscaled(disc);
    if (__ballot(disc < 0x1p-96f)) {  // wave-uniform: no exec-mask save and restore
        asm volatile("");  // a real branch: hipcc would otherwise run the full sqrt for every lane
        region(rrow, reg::kSqrtFallback);
        const float full = __builtin_sqrtf(disc);
        sq = disc < 0x1p-96f ? full : sq;
    }
    const float r1 = div_a(-hb - sq, a, ya);
    // the far root only in waves where some lane rejects the near one (a wave-uniform branch:
    // rays from outside the sphere take the near root; -1.5% VALU at C4, r05_valu_attrib.txt)
    float t = r1;
    if (__ballot(!(r1 > kMinT))) {
        asm volatile("");
        const float r2 = div_a(-hb + sq, a, ya);
        t = r1 > kMinT ? r1 : r2;
    }
    return t;
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

// pair_disc_cc for a camera ray (o = the camera centre) from the camera-relative record
// (TraceParams.cam_rec: oc and cc as pair_disc_cc computes them for that o): the remaining
// operations, in the same order, on the same operands -- the same bits, at half the work.
__device__ __forceinline__ void pair_disc_cam(const v2f dx, const v2f dy, const v2f dz,
                                              const v2f a2, float4 oxy, float4 ozc, v2f& hb,
                                              v2f& cc, v2f& disc) {
    const v2f ocx = {oxy.x, oxy.y}, ocy = {oxy.z, oxy.w}, ocz = {ozc.x, ozc.y};
    cc = (v2f){ozc.z, ozc.w};
    hb = ocx * dx + ocy * dy + ocz * dz;
    disc = hb * hb - a2 * cc;
}

__device__ __forceinline__ void consider(float t, int idx, float& max_t, int& best) {
    // (t, idx) < (max_t, best) lexicographically, as one 64-bit compare of (bits(t), index)
    // (t, max_t > min_t > 0 order as their bits); best < 0 (none yet) counts as index 0, so a
    // t equal to the initial max_t is never taken, as in hit_sphere's strict "<"
    const uint64_t kt = ((uint64_t)__float_as_uint(t) << 32) | (uint32_t)idx;
    const uint64_t km = ((uint64_t)__float_as_uint(max_t) << 32) | (uint32_t)max(best, 0);
    const bool take = (t > kMinT) & (kt < km);
    max_t = take ? t : max_t;
    best = take ? idx : best;
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

struct CullRay {  // one ray's origin, splatted for packed tests
    v2f ox, oy, oz;
};

// One ray prepared for the box test (3), splatted for packed tests.
struct BoxRay {
    v2f ix, iy, iz;  // 1 / d'
    v2f cx, cy, cz;  // -o / d'
    v2f c1, c2;      // gap slack: c1 + K_b c2
};

__device__ __forceinline__ float box_axis(float o, float d, float tau, v2f& i, v2f& c) {
    const float dd = copysignf(fmaxf(fabsf(d), 0x1p-40f), d);
    const float iv = __builtin_amdgcn_rcpf(dd);
    const float co = __builtin_fmaf(-o, iv, tau);  // the plane shift of (4) (tau = 0: none)
    i = (v2f){iv, iv};
    c = (v2f){co, co};
    return fabsf(iv);
}

// ya: recip_a(dot(d, d)), for tau of (4)
__device__ __forceinline__ BoxRay box_ray(const TraceParams& p, const f3 o, const f3 d, float ya) {
    BoxRay r;
    const float on = __builtin_amdgcn_sqrtf(dot(o, o)) + p.box_margin[0];
    const float Q = on * on + p.box_margin[1];
    const float tau = __builtin_amdgcn_sqrtf(3.2e-7f * Q * ya);  // (4)
    const float ax = box_axis(o.x, d.x, tau, r.ix, r.cx), ay = box_axis(o.y, d.y, tau, r.iy, r.cy),
                az = box_axis(o.z, d.z, tau, r.iz, r.cz);
    const float J = 2.002f * fmaxf(fmaxf(ax, ay), az);  // 1.001 J
    const float oinf = fmaxf(fmaxf(fabsf(o.x), fabsf(o.y)), fabsf(o.z));
    const float c1 = J * (3.04e-7f * (p.box_margin[2] + oinf));  // 5.1u
    const float c2 = J * Q;
    r.c1 = (v2f){c1, c1};
    r.c2 = (v2f){c2, c2};
    return r;
}

// The box test's gap for a pair of boxes (TraceParams.cbound: (lox0,lox1,loy0,loy1)
// (loz0,loz1,hix0,hix1) (hiy0,hiy1,hiz0,hiz1) (K0,K1,-,-)): negative when the ray rules the box
// out. (All values finite or +inf, so the gap is never -0 or NaN.)
__device__ __forceinline__ v2f box_gap(const BoxRay& r, float4 b0, float4 b1, float4 b2,
                                       float4 b3) {
    const v2f lox = {b0.x, b0.y}, loy = {b0.z, b0.w}, loz = {b1.x, b1.y};
    const v2f hix = {b1.z, b1.w}, hiy = {b2.x, b2.y}, hiz = {b2.z, b2.w}, K = {b3.x, b3.y};
    const v2f tlx = vfma(lox, r.ix, r.cx), thx = vfma(hix, r.ix, r.cx);
    const v2f tly = vfma(loy, r.iy, r.cy), thy = vfma(hiy, r.iy, r.cy);
    const v2f tlz = vfma(loz, r.iz, r.cz), thz = vfma(hiz, r.iz, r.cz);
    v2f tn, tf;
    tn.x = fmaxf(fmaxf(fminf(tlx.x, thx.x), fminf(tly.x, thy.x)), fminf(tlz.x, thz.x));
    tn.y = fmaxf(fmaxf(fminf(tlx.y, thx.y), fminf(tly.y, thy.y)), fminf(tlz.y, thz.y));
    tf.x = fminf(fminf(fmaxf(tlx.x, thx.x), fmaxf(tly.x, thy.x)), fmaxf(tlz.x, thz.x));
    tf.y = fminf(fminf(fmaxf(tlx.y, thx.y), fmaxf(tly.y, thy.y)), fmaxf(tlz.y, thz.y));
    // (4): the stretch of the line behind -tau does not count
    tn.x = fmaxf(tn.x, 0.0f);
    tn.y = fmaxf(tn.y, 0.0f);
    return vfma(K, r.c2, (tf - tn) + r.c1);
}

// Box test of one pair, wave-uniform: bit 0/1 set when some lane may accept a member of box
// 0/1.
struct BoundPair {
    float4 b0, b1, b2, b3;
};

__device__ __forceinline__ BoundPair load_bound_pair(cfloat4* b) {
    return BoundPair{b[0], b[1], b[2], b[3]};
}

template <bool kStats>
__device__ __forceinline__ uint32_t bound_pair_need(const BoxRay& r, const BoundPair& bp,
                                                    uint32_t& lane_needs, uint32_t& lane_cnt) {
    const v2f g = box_gap(r, bp.b0, bp.b1, bp.b2, bp.b3);
    const bool m0 = !(g.x < 0.0f), m1 = !(g.y < 0.0f);
    const uint64_t n0 = __ballot(m0), n1 = __ballot(m1);
    if constexpr (kStats) {
        lane_needs += __popcll(n0) + __popcll(n1);
        lane_cnt += (uint32_t)m0 + (uint32_t)m1;
    }
    return nonzero(n0) | (nonzero(n1) << 1);
}

// The exact test of one group for every lane (wave-uniform scalar loads of the 80-B record):
// the big-sphere list, tested for every ray ahead of the hierarchy.
__device__ __forceinline__ void exact_group_uniform(cfloat4* rec, const CullRay& r, v2f dx, v2f dy,
                                                    v2f dz, v2f a2, float a, float ya,
                                                    float& max_t, int& best,
                                                    uint32_t* rrow = nullptr, uint32_t rb = 0) {
    const float4 q0 = rec[0], q1 = rec[1], idf = rec[4];
    v2f hb01, cc01, d01, hb23 = {0.f, 0.f}, cc23 = {0.f, 0.f}, d23 = {-1.f, -1.f};
    pair_disc_cc(r.ox, r.oy, r.oz, dx, dy, dz, a2, q0, q1, hb01, cc01, d01);
    // members 2 and 3 only when the group has them (wave-uniform)
    if (__float_as_int(idf.z) >= 0 || __float_as_int(idf.w) >= 0)
        pair_disc_cc(r.ox, r.oy, r.oz, dx, dy, dz, a2, rec[2], rec[3], hb23, cc23, d23);
    const float m4 = fmaxf(fmaxf(d01.x, d01.y), fmaxf(d23.x, d23.y));
    if (__ballot(!(m4 < 0.0f))) {
        region(rrow, rb);
        if (may_hit(hb01.x, cc01.x, d01.x)) {
            region(rrow, rb + 1);
            consider(candidate_t_fast(hb01.x, d01.x, a, ya, rrow), __float_as_int(idf.x), max_t,
                     best);
        }
        if (may_hit(hb01.y, cc01.y, d01.y)) {
            region(rrow, rb + 2);
            consider(candidate_t_fast(hb01.y, d01.y, a, ya, rrow), __float_as_int(idf.y), max_t,
                     best);
        }
        if (may_hit(hb23.x, cc23.x, d23.x)) {
            region(rrow, rb + 3);
            consider(candidate_t_fast(hb23.x, d23.x, a, ya, rrow), __float_as_int(idf.z), max_t,
                     best);
        }
        if (may_hit(hb23.y, cc23.y, d23.y)) {
            region(rrow, rb + 4);
            consider(candidate_t_fast(hb23.y, d23.y, a, ya, rrow), __float_as_int(idf.w), max_t,
                     best);
        }
    }
}

// exact_group_uniform for camera rays, from the group's camera-relative record `crec` (the
// member indices still come from the group record `rec`).
__device__ __forceinline__ void exact_group_uniform_cam(cfloat4* crec, cfloat4* rec, v2f dx,
                                                        v2f dy, v2f dz, v2f a2, float a,
                                                        float ya, float& max_t, int& best,
                                                        uint32_t* rrow = nullptr,
                                                        uint32_t rb = 0) {
    const float4 c0 = crec[0], c1 = crec[1], idf = rec[4];
    v2f hb01, cc01, d01, hb23 = {0.f, 0.f}, cc23 = {0.f, 0.f}, d23 = {-1.f, -1.f};
    pair_disc_cam(dx, dy, dz, a2, c0, c1, hb01, cc01, d01);
    if (__float_as_int(idf.z) >= 0 || __float_as_int(idf.w) >= 0)
        pair_disc_cam(dx, dy, dz, a2, crec[2], crec[3], hb23, cc23, d23);
    const float m4 = fmaxf(fmaxf(d01.x, d01.y), fmaxf(d23.x, d23.y));
    if (__ballot(!(m4 < 0.0f))) {
        region(rrow, rb);
        if (may_hit(hb01.x, cc01.x, d01.x)) {
            region(rrow, rb + 1);
            consider(candidate_t_fast(hb01.x, d01.x, a, ya, rrow), __float_as_int(idf.x), max_t,
                     best);
        }
        if (may_hit(hb01.y, cc01.y, d01.y)) {
            region(rrow, rb + 2);
            consider(candidate_t_fast(hb01.y, d01.y, a, ya, rrow), __float_as_int(idf.y), max_t,
                     best);
        }
        if (may_hit(hb23.x, cc23.x, d23.x)) {
            region(rrow, rb + 3);
            consider(candidate_t_fast(hb23.x, d23.x, a, ya, rrow), __float_as_int(idf.z), max_t,
                     best);
        }
        if (may_hit(hb23.y, cc23.y, d23.y)) {
            region(rrow, rb + 4);
            consider(candidate_t_fast(hb23.y, d23.y, a, ya, rrow), __float_as_int(idf.w), max_t,
                     best);
        }
    }
}

// Stats builds count in `hit_groups` the lanes that need each group (sum over group bounds)
// and in `lane_cnt` the groups this lane needs.
template <bool kStats>
__device__ __forceinline__ void scan_culled(const TraceParams& p, const f3 o, const f3 d,
                                            float& max_t, int& best, uint32_t& groups_tested,
                                            uint32_t& bounds_tested, uint32_t& hit_groups,
                                            uint32_t& lane_cnt) {
    uint32_t node_lanes = 0, node_cnt = 0;
    uint32_t n_groups = 0, n_bounds = 0;
    const float a = dot(d, d);
    CullRay r;
    r.ox = (v2f){o.x, o.x};
    r.oy = (v2f){o.y, o.y};
    r.oz = (v2f){o.z, o.z};
    const BoxRay br = box_ray(p, o, d, recip_a(a));
    const v2f dx = {d.x, d.x}, dy = {d.y, d.y}, dz = {d.z, d.z}, a2 = {a, a};
    cfloat4* bound = (cfloat4*)p.cbound;
    cfloat4* node = (cfloat4*)p.cnode;
    cfloat4* geom = (cfloat4*)p.cgroup;
    for (int gb = 0; gb < p.nbig; ++gb)  // the big spheres, for every ray
        exact_group_uniform(geom + 5 * gb, r, dx, dy, dz, a2, a, recip_a(a), max_t, best);
    n_groups += (uint32_t)p.nbig;
    geom += 5 * p.nbig;           // the hierarchy's groups
    const int ncg = p.ncgroups;  // multiple of 16: whole node pairs
    cfloat4* top = (cfloat4*)p.ctop;
    uint32_t tops = 0;
    for (int base = 0; base < ncg; base += 64) {
        // level 0: the chunk's own bound (tested for two chunks at a time)
        if ((base & 127) == 0) {
            tops = bound_pair_need<false>(br, load_bound_pair(top + 4 * (base >> 7)), node_lanes,
                                          node_cnt);
            n_bounds += 2;
        }
        if (((tops >> ((base >> 6) & 1)) & 1u) == 0) continue;
        // level 1: which of the next (up to) 8 nodes of 8 groups may any lane hit? (the
        // scalar loads run one pair ahead of the tests)
        const int nn = min(8, (ncg - base) >> 3);
        cfloat4* nb = node + 4 * (base >> 4);
        uint32_t nodes = 0;
        BoundPair cur = load_bound_pair(nb);
        for (int j = 0; j < nn; j += 2) {
            const BoundPair nxt = load_bound_pair(nb + 4 * ((j + 2 < nn ? j + 2 : j) >> 1));
            nodes |= bound_pair_need<false>(br, cur, node_lanes, node_cnt) << j;
            cur = nxt;
        }
        n_bounds += (uint32_t)(nn + 8 * __popc(nodes));
        // level 2: which groups of those nodes?
        uint64_t need = 0;
        if (nodes) cur = load_bound_pair(bound + 4 * ((base + 8 * __builtin_ctz(nodes)) >> 1));
        while (nodes) {
            const int j = __builtin_ctz(nodes);
            nodes &= nodes - 1;
            cfloat4* gb = bound + 4 * ((base + 8 * j) >> 1);
            cfloat4* gnext = bound + 4 * ((base + 8 * (nodes ? __builtin_ctz(nodes) : j)) >> 1);
#pragma unroll
            for (int k = 0; k < 8; k += 2) {
                const BoundPair nxt = load_bound_pair(k + 2 < 8 ? gb + 4 * ((k + 2) >> 1) : gnext);
                need |= (uint64_t)bound_pair_need<kStats>(br, cur, hit_groups, lane_cnt)
                        << (8 * j + k);
                cur = nxt;
            }
        }
        // the exact hit_sphere test on the groups that survived (next group prefetched)
        n_groups += (uint32_t)__popcll(need);
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
    tally(groups_tested, 2u * n_groups);  // in half-groups
    tally(bounds_tested, n_bounds);
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

// Sign of the box gap for both boxes of a pair: set (negative) when this lane rules the box
// out. Pushed high element first.
__device__ __forceinline__ uint32_t push_bound_pair(uint32_t acc, const BoxRay& r, float4 b0,
                                                    float4 b1, float4 b2, float4 b3) {
    const v2f D = box_gap(r, b0, b1, b2, b3);
    return push_sign(push_sign(acc, D.y), D.x);
}

// Box test of a group pair in the near/far layout (TraceParams.cbound_nf). For inv = 1/d' > 0
// the exact products order lo*inv <= hi*inv and rounding is monotone, so fma(lo, inv, c) <=
// fma(hi, inv, c): box_gap's per-axis min / max are the lo / hi plane when inv > 0 and the hi / lo
// plane when inv < 0 (d' is never 0). Each axis stores (lo, hi, lo), so the near plane sits at
// byte 8 * sign(inv) of the axis and the far plane 8 bytes after it: one per-lane address per
// axis, one ds_read2_b64 per axis and pair. The gap is box_gap's value (at most the sign of a
// zero tf - tn differs, and adding the slack c1 >= +0 gives the same sum for either zero), for
// one v_max3 + one v_min3 per box instead of 3 min + 3 max + max3 + min3.
struct NearFarAddr {
    const char* x;  // near plane of axis x of pair 0 (far: + 8 bytes)
    const char* y;
    const char* z;
    const char* k;  // (K0, K1) of pair 0
};

__device__ __forceinline__ NearFarAddr near_far_addr(const float4* pairs, float ix, float iy,
                                                     float iz) {
    const char* b = reinterpret_cast<const char*>(pairs);
    NearFarAddr a;
    a.x = b + ((__float_as_uint(ix) >> 31) << 3);
    a.y = b + 24 + ((__float_as_uint(iy) >> 31) << 3);
    a.z = b + 48 + ((__float_as_uint(iz) >> 31) << 3);
    a.k = b + 72;
    return a;
}

__device__ __forceinline__ v2f ld2(const char* p) {
    const float2 v = *reinterpret_cast<const float2*>(p);
    return (v2f){v.x, v.y};
}

__device__ __forceinline__ uint32_t push_bound_pair_nf(uint32_t acc, const BoxRay& r,
                                                       const NearFarAddr& a, int off) {
    const v2f tnx = vfma(ld2(a.x + off), r.ix, r.cx), tfx = vfma(ld2(a.x + off + 8), r.ix, r.cx);
    const v2f tny = vfma(ld2(a.y + off), r.iy, r.cy), tfy = vfma(ld2(a.y + off + 8), r.iy, r.cy);
    const v2f tnz = vfma(ld2(a.z + off), r.iz, r.cz), tfz = vfma(ld2(a.z + off + 8), r.iz, r.cz);
    v2f tn, tf;
    tn.x = fmaxf(fmaxf(tnx.x, tny.x), tnz.x);
    tn.y = fmaxf(fmaxf(tnx.y, tny.y), tnz.y);
    tf.x = fminf(fminf(tfx.x, tfy.x), tfz.x);
    tf.y = fminf(fminf(tfx.y, tfy.y), tfz.y);
    tn.x = fmaxf(tn.x, 0.0f);  // (4), as box_gap
    tn.y = fmaxf(tn.y, 0.0f);
    const v2f D = vfma(ld2(a.k + off), r.c2, (tf - tn) + r.c1);
    return push_sign(push_sign(acc, D.y), D.x);
}

// Sign bit set when a member may be accepted: disc >= 0 and (hb < 0 or cc < 0), by sign bits
// (a -0 hb only adds a candidate that the exact test then rejects; disc is never -0).
__device__ __forceinline__ float hit_sign(float hb, float cc, float disc) {
    return __uint_as_float((__float_as_uint(hb) | __float_as_uint(cc)) & ~__float_as_uint(disc));
}

// ---- flattened scan (variant CULL_FLAT) ------------------------------------------------------
// The per-lane scan runs each level as many wave passes as its busiest lane needs (twice the
// mean). Here the work items of the per-lane levels and of the root evaluation are kept as
// four per-wave stacks in LDS and dealt to the wave's live lanes a full wave at a time, each
// lane working on another lane's ray (fetched with ds_bpermute):
//   chunk (owner, chunk)               -> tests the chunk's <= 8 node bounds -> node entries
//   node  (owner, node)                -> tests the node's 8 group bounds -> group entries
//   group (owner, group)               -> exact test of the 4 members     -> candidate entries
//   cand  (owner, group, member)       -> the accepted root, into the owner's key
// Entries are pushed at a wave prefix of the lanes' counts (their order never matters; stack
// heights are wave-uniform, in SGPRs) and carried from chunk to chunk; only the segment's last
// passes run partly empty. (A per-lane LDS atomic add on the height instead serialises on its
// one address: 9x the LDS bank conflicts of the per-lane scan, 9% slower overall.) Every owner's
// (t, sphere index) minimum is an LDS 64-bit word updated with ds_min_u64: the lexicographic
// minimum of (t, index) is what `consider` computes, since t > 0 orders like its bit pattern.
// A pass pushes onto the next stack only while that stack holds < nact <= 64 entries (full
// passes run deepest stack first; the final drain's partial passes run top-down), which bounds
// every stack: < 64 left over + at most 8 x 64 (node, group) or 4 x 64 (cand) pushed by one pass;
// chunk entries (one per lane and chunk) are pushed between drains, onto < 64 left over.
// (Round 2: the chunk level was wave-uniform -- every lane tested the nodes of every chunk some
// lane needed, with per-lane min/max box tests on scalar-loaded boxes; as passes the nodes are
// tested only for the lanes that need the chunk, by the near/far box test.)
constexpr int kPendSky = -2;  // trace_impl's pend_best for a deferred sky segment
constexpr int kChunkCap = 128;
constexpr int kNodeCap = 576;
constexpr int kGroupCap = 576;
constexpr int kCandCap = 320;

// Stack entries, by format kFmt:
//   0 (narrow8, the LDS-table kernel, <= 256 groups): 16-bit owner << 8 | index, and 16-bit
//     candidate entries (node/group entry) << 2 | member;
//   1 (narrow10, the boxes-in-LDS kernel, <= 1024 groups): 16-bit owner << 10 | index,
//     32-bit candidate entries;
//   2 (wide, the global-table kernel, any size): 32-bit owner << 24 | index and candidates.
template <int kFmt>
struct FlatFmt {
    using entry_t = typename std::conditional<kFmt == 2, uint32_t, uint16_t>::type;
    using cand_t = typename std::conditional<kFmt == 0, uint16_t, uint32_t>::type;
    static constexpr int kShift = kFmt == 2 ? 24 : kFmt == 1 ? 10 : 8;  // owner field
    static constexpr uint32_t kMask = (1u << kShift) - 1u;
};

template <int kFmt, bool kChunks = true>
struct WaveScratch {
    using entry_t = typename FlatFmt<kFmt>::entry_t;
    static constexpr bool kHasChunks = kChunks;
    unsigned long long key[64];  // per owner lane: (bits(t) << 32) | sphere index
    uint32_t work[2];            // issued-work tallies of the flat scan: half-groups, box tests
    typename FlatFmt<kFmt>::cand_t cand[kCandCap];  // group entry << 2 | member
    entry_t group[kGroupCap];    // owner << kShift | group
    entry_t node[kNodeCap];      // owner << kShift | node
    entry_t chunk[kChunks ? kChunkCap : 0];  // owner << kShift | chunk (64 groups)
};
static_assert(sizeof(WaveScratch<0, false>) == kWaveScratchBytes8, "host LDS size");  // 3464
static_assert(sizeof(WaveScratch<1>) == kWaveScratchBytes, "host LDS size");
static_assert(sizeof(WaveScratch<2>) == kWaveScratchBytesWide, "host LDS size");

// The flat scans' hierarchy group records, 80 B each: four pair-SoA float4s + the members'
// world[] indices. Global records (kGRec, TraceParams.cgroup): the indices as int bits. LDS
// records: the indices as uint16 in the first 8 B of the fifth float4 (the 80-B stride starts
// 16 consecutive records on 16 different bank quadruples, so the ds_read_b128 of a 16-lane group
// reading different groups is conflict-free; a 64-B stride gave four).
template <bool kGRec>
struct GroupTab {
    const float4* geom;
    __device__ __forceinline__ const float4* rec(uint32_t gi) const { return geom + 5u * gi; }
    __device__ __forceinline__ int index(uint32_t gi, uint32_t s) const {
        if constexpr (kGRec) {
            const float4 idf = geom[5u * gi + 4u];
            return __float_as_int(s == 0 ? idf.x : s == 1 ? idf.y : s == 2 ? idf.z : idf.w);
        } else {
            return (int)reinterpret_cast<const uint16_t*>(geom + 5u * gi + 4u)[s];
        }
    }
};

__device__ __forceinline__ unsigned long long pack_hit(float t, int idx) {
    return ((unsigned long long)__float_as_uint(t) << 32) | (uint32_t)idx;
}

// Exclusive prefix over the active lanes of a per-lane count c < 2^kBits, and the wave total.
// With every lane active: an inclusive DPP scan (row_shr 1/2/4/8, row_bcast 15/31; 8 VALU).
// Otherwise (the drain at the end of the grid, where finished lanes are masked off and DPP
// would read their stale registers): bit-sliced ballots, ~5 VALU per bit.
template <int kBits>
__device__ __forceinline__ uint32_t wave_prefix(uint32_t c, uint32_t& total,
                                                uint32_t* rrow = nullptr) {
    if (__builtin_amdgcn_read_exec() == ~0ull) {
        int x = (int)c;
        x += __builtin_amdgcn_update_dpp(0, x, 0x111, 0xf, 0xf, false);  // row_shr:1
        x += __builtin_amdgcn_update_dpp(0, x, 0x112, 0xf, 0xf, false);  // row_shr:2
        x += __builtin_amdgcn_update_dpp(0, x, 0x114, 0xf, 0xf, false);  // row_shr:4
        x += __builtin_amdgcn_update_dpp(0, x, 0x118, 0xf, 0xf, false);  // row_shr:8
        x += __builtin_amdgcn_update_dpp(0, x, 0x142, 0xa, 0xf, false);  // row_bcast:15
        x += __builtin_amdgcn_update_dpp(0, x, 0x143, 0xc, 0xf, false);  // row_bcast:31
        total = (uint32_t)__builtin_amdgcn_readlane(x, 63);
        return (uint32_t)x - c;
    }
    region(rrow, reg::kPrefixSlow);
    uint32_t pre = 0, tot = 0;
#pragma unroll
    for (int b = 0; b < kBits; ++b) {
        const uint64_t m = __ballot((c >> b) & 1u);
        pre += lanes_below(m) << b;
        tot += (uint32_t)__popcll(m) << b;
    }
    total = tot;
    return pre;
}

// Maximum over the active lanes of v < 2^kBits, wave-uniform: one compare per bit (ballots)
// instead of a shuffle reduction.
template <int kBits>
__device__ __forceinline__ uint32_t wave_max_small(uint32_t v) {
    uint32_t m = 0;
#pragma unroll
    for (int b = kBits - 1; b >= 0; --b)
        if (__ballot(v >= (m | (1u << b)))) m |= 1u << b;
    return m;
}

// v of lane src_x4 / 4 (ds_bpermute; the source lane is live)
__device__ __forceinline__ float from_lane(int src_x4, float v) {
    return __int_as_float(__builtin_amdgcn_ds_bpermute(src_x4, __float_as_int(v)));
}

struct FlatRay {  // this lane's ray, as the passes fetch it
    float ox, oy, oz, dx, dy, dz, a, ya;
    BoxRay br;
};

// One pass over the top min(n, nact) entries of a stack (n wave-uniform). kind 0: cand,
// 1: group, 2: node. Lanes ranked past the entries run on their own ray and push nothing.
// kKind 0: cand, 1: group, 2: node. n: this stack's height; pushed: the height of the stack
// this pass pushes onto (group for node passes, cand for group passes).
template <int kKind, int kFmt, bool kGRec, uint32_t kNS, class WS>
__device__ __forceinline__ void flat_pass(uint32_t& n, uint32_t& pushed, uint32_t nact,
                                          uint32_t rank, uint32_t lane, WS* ws,
                                          const float4* tbound, const float4* tnode, uint32_t ncg,
                                          const GroupTab<kGRec>& tg, const FlatRay& my,
                                          uint32_t* rrow = nullptr) {
    using F = FlatFmt<kFmt>;
    using entry_t = typename F::entry_t;
    const uint32_t m = min(n, nact), top = n - m;
    n = top;
    const bool act = rank < m;
    if constexpr (kKind == 2 || kKind == 3) {  // node: the 8 group bounds of (owner, node);
                                               // chunk: the <= 8 node bounds of (owner, chunk)
        uint32_t e = lane << F::kShift;
        if (act) {
            if constexpr (kKind == 2)
                e = ws->node[top + rank];
            else
                e = ws->chunk[top + rank];
        }
        const int src = (int)(e >> F::kShift) << 2;
        BoxRay r;
        const float ix = from_lane(src, my.br.ix.x), iy = from_lane(src, my.br.iy.x),
                    iz = from_lane(src, my.br.iz.x);
        const float cx = from_lane(src, my.br.cx.x), cy = from_lane(src, my.br.cy.x),
                    cz = from_lane(src, my.br.cz.x);
        const float c1 = from_lane(src, my.br.c1.x), c2 = from_lane(src, my.br.c2.x);
        r.ix = (v2f){ix, ix};
        r.iy = (v2f){iy, iy};
        r.iz = (v2f){iz, iz};
        r.cx = (v2f){cx, cx};
        r.cy = (v2f){cy, cy};
        r.cz = (v2f){cz, cz};
        r.c1 = (v2f){c1, c1};
        r.c2 = (v2f){c2, c2};
        // 4 pairs x 80 B: a node's 8 groups, or a chunk's 8 nodes (padded past the last one)
        const float4* gb = (kKind == 2 ? tbound : tnode) + kNS * (e & F::kMask);
        const NearFarAddr na = near_far_addr(gb, ix, iy, iz);
        uint32_t gout = 0;
#pragma unroll
        for (int k = 3; k >= 0; k--) gout = push_bound_pair_nf(gout, r, na, 80 * k);
        uint32_t valid = 0xffu;
        if constexpr (kKind == 3)  // the last chunk may hold fewer than 8 nodes
            valid = (1u << min(8u, (ncg >> 3) - 8u * (e & F::kMask))) - 1u;
        uint32_t need = act ? (~gout & valid) : 0u;
        uint32_t tot;
        uint32_t pos = pushed + wave_prefix<4>((uint32_t)__popc(need), tot, rrow);
        pushed += tot;
        if (need) {
            const uint32_t tag = (e & ~F::kMask) | ((e & F::kMask) << 3);
            do {
                region(rrow, reg::kPushNode);
                const uint32_t k = (uint32_t)__builtin_ctz(need);
                need &= need - 1;
                if constexpr (kKind == 2)
                    ws->group[pos++] = (entry_t)(tag | k);
                else
                    ws->node[pos++] = (entry_t)(tag | k);
            } while (need);
        }
    } else if constexpr (kKind == 1) {  // group: exact test of the 4 members for the owner's ray
        const uint32_t e = act ? (uint32_t)ws->group[top + rank] : (lane << F::kShift);
        const int src = (int)(e >> F::kShift) << 2;
        const float ox = from_lane(src, my.ox), oy = from_lane(src, my.oy), oz = from_lane(src, my.oz);
        const float dx = from_lane(src, my.dx), dy = from_lane(src, my.dy), dz = from_lane(src, my.dz);
        const float a = from_lane(src, my.a);
        const float4* g = tg.rec(e & F::kMask);
        const float4 q0 = g[0], q1 = g[1], q2 = g[2], q3 = g[3];
        const v2f vox = {ox, ox}, voy = {oy, oy}, voz = {oz, oz};
        const v2f vdx = {dx, dx}, vdy = {dy, dy}, vdz = {dz, dz}, a2 = {a, a};
        v2f hb01, cc01, d01, hb23, cc23, d23;
        pair_disc_cc(vox, voy, voz, vdx, vdy, vdz, a2, q0, q1, hb01, cc01, d01);
        pair_disc_cc(vox, voy, voz, vdx, vdy, vdz, a2, q2, q3, hb23, cc23, d23);
        uint32_t hits = push_sign(0u, hit_sign(hb23.y, cc23.y, d23.y));
        hits = push_sign(hits, hit_sign(hb23.x, cc23.x, d23.x));
        hits = push_sign(hits, hit_sign(hb01.y, cc01.y, d01.y));
        hits = push_sign(hits, hit_sign(hb01.x, cc01.x, d01.x));
        hits = act ? hits : 0u;
        uint32_t tot;
        uint32_t pos = pushed + wave_prefix<3>((uint32_t)__popc(hits), tot, rrow);
        pushed += tot;
        if (hits) {
            const uint32_t tag = e << 2;
            do {
                region(rrow, reg::kPushGroup);
                const uint32_t s = (uint32_t)__builtin_ctz(hits);
                hits &= hits - 1;
                ws->cand[pos++] = (typename F::cand_t)(tag | s);
            } while (hits);
        }
    } else {  // cand: the member's root (its hb, cc, disc recomputed as the packed test did)
        const uint32_t e = act ? ws->cand[top + rank] : (lane << (F::kShift + 2));
        const int src = (int)(e >> (F::kShift + 2)) << 2;
        const float ox = from_lane(src, my.ox), oy = from_lane(src, my.oy), oz = from_lane(src, my.oz);
        const float dx = from_lane(src, my.dx), dy = from_lane(src, my.dy), dz = from_lane(src, my.dz);
        const float a = from_lane(src, my.a), ya = from_lane(src, my.ya);
        const uint32_t s = e & 3u;
        const uint32_t gi = (e >> 2) & F::kMask;
        const float4* g = tg.rec(gi);
        const float4 xy = g[(s >> 1) * 2], zr = g[(s >> 1) * 2 + 1];
        const bool hi = (s & 1u) != 0;
        const float cx = hi ? xy.y : xy.x, cy = hi ? xy.w : xy.z;
        const float cz = hi ? zr.y : zr.x, r2 = hi ? zr.w : zr.z;
        const float ocx = ox - cx, ocy = oy - cy, ocz = oz - cz;
        const float hb = ocx * dx + ocy * dy + ocz * dz;
        const float cc = (ocx * ocx + ocy * ocy + ocz * ocz) - r2;
        const float disc = hb * hb - a * cc;
        const float t = candidate_t_fast(hb, disc, a, ya);
        if (act && t > kMinT && t < kInfinity)
            atomicMin(&ws->key[e >> (F::kShift + 2)], pack_hit(t, tg.index(gi, s)));
    }
}

// Runs passes while a stack holds at least `th` entries (th = nact: full passes only; 1: drain).
// Stats builds: wave clock ticks per phase (s_memtime, wave-uniform).
struct PhaseTicks {
    uint64_t scan = 0, levels = 0, node = 0, group = 0, cand = 0, cand_passes = 0, big = 0,
             push = 0, shade = 0, fetch = 0;
    uint64_t pass_entries = 0, pass_lanes = 0, partial_passes = 0, passes = 0;
    uint64_t cam = 0;  // the camera fast trace with its shading
    // camera fast trace occupancy: entries, camera lanes, live lanes, listed-loop trips and
    // lane sum, root-loop trips and lane sum; main shading hit lanes
    uint64_t cam_entries = 0, cam_lanes = 0, cam_live = 0, list_trips = 0, list_sum = 0,
             root_trips = 0, root_sum = 0, shade_hits = 0;
    // the loop top: wave ticks in the retire, wave-iterations running the fetch loop, block
    // fetches, items started, wave-iterations running the retire, quanta retired (lanes)
    uint64_t retire = 0, fetch_iters = 0, blk_fetches = 0, items_cur = 0, retire_iters = 0,
             quanta = 0;
};

__device__ __forceinline__ uint64_t ticks() { return __builtin_amdgcn_s_memtime(); }

struct FlatStacks {  // wave-uniform stack heights
    uint32_t cand, group, node, chunk;
};

template <bool kStats, int kFmt, bool kGRec, uint32_t kNS, class WS>
__device__ __forceinline__ void flat_drain(uint32_t th, uint32_t nact, uint32_t rank, uint32_t lane,
                                           WS* ws, FlatStacks& h,
                                           const float4* tbound, const float4* tnode, uint32_t ncg,
                                           const GroupTab<kGRec>& tg, const FlatRay& my,
                                           uint32_t& n_groups, uint32_t& n_bounds,
                                           PhaseTicks& pt, uint32_t* rrow = nullptr) {
    uint32_t nc = h.cand, ng = h.group, nn = h.node, nk = h.chunk;
    for (;;) {
        __builtin_amdgcn_wave_barrier();  // the entries were written by other lanes
        region(rrow, reg::kDrainTrip);
        uint64_t t0 = 0;
        if constexpr (kStats) {
            t0 = ticks();
            const uint32_t n = nc >= nact ? nc : ng >= nact ? ng : nn >= nact ? nn
                             : nk >= nact ? nk
                             : th == 1u ? (nk ? nk : nn ? nn : ng ? ng : nc) : 0u;
            if (n) {
                pt.pass_entries += min(n, nact);
                pt.pass_lanes += nact;
                pt.partial_passes += n < nact;
                ++pt.passes;
            }
        }
        // full passes first, deepest stack first; then (final drain only) the partial passes
        // top-down, chunks before nodes before groups before candidates, so that each level's
        // remainder joins the next level's before that one runs: ~3 partial passes per segment
        // instead of a cascade. A pass onto a stack runs only while that stack holds < nact <= 64
        // entries, which keeps the caps (see kNodeCap).
        int kind = -1;
        if (nc >= nact) kind = 0;
        else if (ng >= nact) kind = 1;
        else if (nn >= nact) kind = 2;
        else if (nk >= nact) kind = 3;
        else if (th == 1u) kind = nk ? 3 : nn ? 2 : ng ? 1 : nc ? 0 : -1;
        if (kind == 0) {
            region(rrow, reg::kPassCand);
            flat_pass<0, kFmt, kGRec, kNS>(nc, nc, nact, rank, lane, ws, tbound, tnode, ncg, tg, my,
                                           rrow);
            if constexpr (kStats) {
                pt.cand += ticks() - t0;
                ++pt.cand_passes;
            }
        } else if (kind == 1) {
            region(rrow, reg::kPassGroup);
            ++n_groups;
            flat_pass<1, kFmt, kGRec, kNS>(ng, nc, nact, rank, lane, ws, tbound, tnode, ncg, tg, my,
                                           rrow);
            if constexpr (kStats) pt.group += ticks() - t0;
        } else if (kind == 2) {
            region(rrow, reg::kPassNode);
            n_bounds += 8;
            flat_pass<2, kFmt, kGRec, kNS>(nn, ng, nact, rank, lane, ws, tbound, tnode, ncg, tg, my,
                                           rrow);
            if constexpr (kStats) pt.node += ticks() - t0;
        } else if (kind == 3) {
            if constexpr (WS::kHasChunks) {  // (nk stays 0 without the chunk stack)
                region(rrow, reg::kPassChunk);
                n_bounds += 8;
                flat_pass<3, kFmt, kGRec, kNS>(nk, nn, nact, rank, lane, ws, tbound, tnode, ncg,
                                                tg, my, rrow);
                if constexpr (kStats) pt.levels += ticks() - t0;
            }
        } else {
            break;
        }
    }
    h.cand = nc;
    h.group = ng;
    h.node = nn;
    h.chunk = nk;
}

// kChunks: the chunk level as per-lane chunk passes over the near/far node boxes `tnode` (many
// chunks: the stress scene), else wave-uniform node tests on scalar-loaded boxes (two chunks:
// the final scene).
template <bool kStats, int kFmt, bool kGRec, bool kChunks, uint32_t kNS, class WS>
__device__ __forceinline__ void scan_culled_flat(const TraceParams& p, const float4* tbound,
                                                 const float4* tnode,
                                                 const GroupTab<kGRec>& tg, WS* ws,
                                                 const f3 o, const f3 d, bool primary,
                                                 uint32_t item, float& max_t, int& best,
                                                 uint32_t& groups_tested, uint32_t& bounds_tested,
                                                 PhaseTicks& pt, uint32_t* rrow = nullptr) {
    uint64_t t_in = 0;
    if constexpr (kStats) t_in = ticks();
    // the camera-ray list record, loaded ahead of the big list so its latency overlaps it
    uint32_t inf = 15u;
    if (primary && p.prim_info != nullptr)  // the list of the item's 4x4 quarter (slot 8 y + x)
        inf = p.prim_info[2u * ((item >> 6) * 4u + (((item >> 5) & 1u) << 1) + ((item >> 2) & 1u))];
    FlatRay my;
    my.ox = o.x;
    my.oy = o.y;
    my.oz = o.z;
    my.dx = d.x;
    my.dy = d.y;
    my.dz = d.z;
    my.a = dot(d, d);
    my.ya = recip_a(my.a);
    my.br = box_ray(p, o, d, my.ya);
    const BoxRay& br = my.br;
    CullRay r;
    r.ox = (v2f){o.x, o.x};
    r.oy = (v2f){o.y, o.y};
    r.oz = (v2f){o.z, o.z};
    {
        const v2f dx = {d.x, d.x}, dy = {d.y, d.y}, dz = {d.z, d.z}, a2 = {my.a, my.a};
        for (int gb = 0; gb < p.nbig; ++gb)  // the big spheres, for every ray (scalar loads)
            exact_group_uniform((cfloat4*)p.cgroup + 5 * gb, r, dx, dy, dz, a2, my.a, my.ya, max_t,
                                best, rrow, reg::kMainBig);
    }
    if constexpr (kStats) pt.big += ticks() - t_in;
    uint32_t n_bounds = 0, n_groups = (uint32_t)p.nbig;
    const uint32_t lane = threadIdx.x & 63u;
    // finished lanes are masked off for the whole scan: entries go to the live lanes by rank
    const uint64_t live = __ballot(1);
    const uint32_t nact = (uint32_t)__popcll(live), rank = lanes_below(live);
    ws->key[lane] = pack_hit(max_t, best);
    FlatStacks h = {0u, 0u, 0u, 0u};
    // A camera ray (primary) whose tile has a group list (primary.cpp) pushes those groups
    // straight onto the group stack and skips the chunk and node levels: the list holds every
    // group such a ray may need (at most 8 per lane: at most 512 entries on the empty stack).
    const bool listed = (inf & 15u) != 15u;
    const uint32_t lcnt = listed ? inf & 15u : 0u, loff = inf >> 4;
    if (__ballot(lcnt != 0u)) {  // the stack height stays wave-uniform: prefix over all lanes
        region(rrow, reg::kListed);
        uint32_t tot;
        uint32_t pos = wave_prefix<4>(lcnt, tot, rrow);
        h.group = tot;
        const uint16_t* ids = p.prim_ids + loff;
        for (uint32_t k = 0; k < lcnt; ++k) {
            region(rrow, reg::kListedTrip);
            ws->group[pos++] =
                (typename FlatFmt<kFmt>::entry_t)((lane << FlatFmt<kFmt>::kShift) | ids[k]);
        }
    }
    cfloat4* node = (cfloat4*)p.cnode;
    cfloat4* top = (cfloat4*)p.ctop;
    const int ncg = p.ncgroups;
    uint32_t tops = 0;
    for (int base = 0;; base += 64) {
        uint32_t th = 1u;  // past the last chunk: drain everything
        if (base < ncg) {
            region(rrow, reg::kLevelChunk);
            th = nact;
            uint64_t t0 = 0;
            if constexpr (kStats) t0 = ticks();
            // level 0, wave-uniform: the chunk's own bound (two chunks per test), per-lane bits
            if ((base & 127) == 0) {
                region(rrow, reg::kLevelTop);
                const BoundPair tp = load_bound_pair(top + 4 * (base >> 7));
                tops = ~push_bound_pair(0u, br, tp.b0, tp.b1, tp.b2, tp.b3) & 3u;
                n_bounds += 2;
            }
            const bool in_chunk = !listed && ((tops >> ((base >> 6) & 1)) & 1u) != 0;
            const uint64_t want = __ballot(in_chunk);
            if (want == 0) continue;
            region(rrow, reg::kLevelNodes);
            if constexpr (kChunks) {
            // level 1 (many chunks): a chunk entry per lane whose ray may meet the chunk; chunk
            // passes test its nodes for that lane alone
            if (in_chunk)
                ws->chunk[h.chunk + lanes_below(want)] = (typename FlatFmt<kFmt>::entry_t)(
                    (lane << FlatFmt<kFmt>::kShift) | ((uint32_t)base >> 6));
            h.chunk += (uint32_t)__popcll(want);
            if constexpr (kStats) pt.push += ticks() - t0;
            } else {
            // level 1 (LDS tables: two chunks at the final scene), wave-uniform: nodes of this
            // chunk, per-lane bits -> node entries
            const int nn = min(8, (ncg - base) >> 3);
            uint32_t out = 0;
            {  // near/far planes from the LDS copy of the chunk's node boxes, by the ray's signs
                const NearFarAddr na = near_far_addr(tnode + kNS * ((uint32_t)base >> 6),
                                                     br.ix.x, br.iy.x, br.iz.x);
#pragma unroll
                for (int k = 3; k >= 0; k--) out = push_bound_pair_nf(out, br, na, 80 * k);
                out &= (1u << nn) - 1u;
            }
            n_bounds += (uint32_t)nn;
            uint32_t nodes = in_chunk ? ~out & ((1u << nn) - 1u) : 0u;
            if constexpr (kStats) {
                const uint64_t t1 = ticks();
                pt.levels += t1 - t0;
                t0 = t1;
            }
            uint32_t tot;
            uint32_t pos = h.node + wave_prefix<4>((uint32_t)__popc(nodes), tot, rrow);
            h.node += tot;
            if (nodes) {
                const uint32_t tag = (lane << FlatFmt<kFmt>::kShift) | ((uint32_t)base >> 3);
                do {
                    region(rrow, reg::kPushLevel);
                    const uint32_t j = (uint32_t)__builtin_ctz(nodes);
                    nodes &= nodes - 1;
                    ws->node[pos++] = (typename FlatFmt<kFmt>::entry_t)(tag | j);
                } while (nodes);
            }
            if constexpr (kStats) pt.push += ticks() - t0;
            }
        }
        flat_drain<kStats, kFmt, kGRec, kNS>(th, nact, rank, lane, ws, h, tbound, tnode,
                                         (uint32_t)ncg, tg, my, n_groups, n_bounds, pt, rrow);
        if (base >= ncg) break;
    }
    __builtin_amdgcn_wave_barrier();
    const unsigned long long k = ws->key[lane];
    max_t = __uint_as_float((uint32_t)(k >> 32));
    best = (int)(uint32_t)k;
    (void)groups_tested;
    (void)bounds_tested;
    tally_lds(&ws->work[1], __builtin_amdgcn_readfirstlane(n_bounds));
    tally_lds(&ws->work[0], 2u * __builtin_amdgcn_readfirstlane(n_groups));  // half-groups
}

template <bool kStats>
__device__ __forceinline__ void scan_culled_lane(const TraceParams& p, const float4* tbound,
                                                 const float4* tgroup, const f3 o, const f3 d,
                                                 float& max_t, int& best,
                                                 uint32_t& groups_tested,
                                                 uint32_t& bounds_tested, uint32_t& lane_cnt,
                                                 uint32_t& rounds) {
    const float a = dot(d, d);
    CullRay r;
    r.ox = (v2f){o.x, o.x};
    r.oy = (v2f){o.y, o.y};
    r.oz = (v2f){o.z, o.z};
    const BoxRay br = box_ray(p, o, d, recip_a(a));
    const v2f dx = {d.x, d.x}, dy = {d.y, d.y}, dz = {d.z, d.z}, a2 = {a, a};
    cfloat4* node = (cfloat4*)p.cnode;
    cfloat4* top = (cfloat4*)p.ctop;
    const int ncg = p.ncgroups;
    for (int gb = 0; gb < p.nbig; ++gb)  // the big spheres, for every ray (scalar loads)
        exact_group_uniform((cfloat4*)p.cgroup + 5 * gb, r, dx, dy, dz, a2, a, recip_a(a), max_t,
                            best);
    // per-segment pass counters, wave-uniform: kept in SGPRs, folded into the 64-bit totals once
    uint32_t n_bounds = 0, n_groups = (uint32_t)p.nbig;
    uint32_t tops = 0;
    for (int base = 0; base < ncg; base += 64) {
        // level 0, wave-uniform: the chunk's own bound (two chunks per test), per-lane bits
        if ((base & 127) == 0) {
            const BoundPair tp = load_bound_pair(top + 4 * (base >> 7));
            tops = ~push_bound_pair(0u, br, tp.b0, tp.b1, tp.b2, tp.b3) & 3u;
            n_bounds += 2;
        }
        const bool in_chunk = ((tops >> ((base >> 6) & 1)) & 1u) != 0;
        if (__ballot(in_chunk) == 0) continue;
        // level 1, wave-uniform: nodes of this chunk, per-lane bits
        const int nn = min(8, (ncg - base) >> 3);
        cfloat4* nb = node + 4 * (base >> 4);
        // sign bits pushed from the last node down, so bit j ends up = node j ruled out
        uint32_t out = 0;
        BoundPair cur = load_bound_pair(nb + 4 * ((nn - 2) >> 1));
        for (int j = nn - 2; j >= 0; j -= 2) {
            const BoundPair nxt = load_bound_pair(nb + 4 * ((j >= 2 ? j - 2 : j) >> 1));
            out = push_bound_pair(out, br, cur.b0, cur.b1, cur.b2, cur.b3);
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
                const float4* gb = tbound + 4 * (base >> 1) + __umul24((uint32_t)j, 16u);
                uint32_t gout = 0;
#pragma unroll
                for (int k = 3; k >= 0; k--) {
                    gout = push_bound_pair(gout, br, gb[4 * k], gb[4 * k + 1], gb[4 * k + 2],
                                           gb[4 * k + 3]);
                }
                need |= (uint64_t)(~gout & 0xffu) << (8 * j);
            }
        }
        if constexpr (kStats) lane_cnt += (uint32_t)__popcll(need);
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
    }
    tally(bounds_tested, __builtin_amdgcn_readfirstlane(n_bounds));
    tally(groups_tested, 2u * __builtin_amdgcn_readfirstlane(n_groups));  // half-groups
}

// ---- Accumulation ring ---------------------------------------------------------------------
// Each wave keeps the chunk sums of its current blocks' pixels in LDS: a ring of 32-B entries
// (pixel, three double sums). A block (64 items: all chunks of a few pixels in chunk-minor order)
// takes the next entries of the ring for its pixels, flushing what they held -- partial sums of
// an older block's pixels -- to the pixels' global sums with one f64 atomic per channel; a
// finished item adds its quantized chunk sums to its pixel's entry with LDS atomics (ds_add_f64)
// if the entry still holds that pixel, else straight to the global sums as before. The sums are
// integers below 2^53 (vcrt_math.h "Accumulation"), so every partition of the additions gives
// the same exact total: the image bits do not depend on which additions went through LDS.
// NaN chunk sums add NaN either way. Each wave flushes its ring before it ends.
struct RingEntry {
    uint32_t q;  // local pixel index, ~0: none
    uint32_t pad;
    double s[3];
};
static_assert(sizeof(RingEntry) == 32, "host LDS size");
constexpr uint32_t kQMask = (1u << kRingQBits) - 1u;  // a lane's pixel index without the entry

__device__ __forceinline__ void ring_flush(RingEntry& e, double* accum) {
    if (e.q != ~0u) {
        double* g = accum + 4u * e.q;
        // exact zeros add nothing (+0 + -0 = +0: the sums start at +0); one channel at a time
        // (few registers: this runs in the block fetch, where the whole lane state is live)
#pragma unroll 1
        for (int c = 0; c < 3; ++c) {
            const double v = e.s[c];
            if (v != 0.0) atomicAdd(g + c, v);
        }
    }
}

// A ring block's entry for pixel slot `slot` of local tile lt at tile (txy & 0xffff, txy >> 16):
// flushes the entry's old sums, then holds that pixel with zero sums.
__device__ __forceinline__ void ring_claim(RingEntry* ring, uint32_t ei, uint32_t rn,
                                                     double* accum, uint32_t slot, uint32_t lt,
                                                     uint32_t txy, uint32_t width,
                                                     uint32_t height) {
    if (ei >= rn) ei -= rn;
    RingEntry& re = ring[ei];
    ring_flush(re, accum);
    const uint32_t px = 8u * (txy & 0xffffu) + (slot & 7u), py = 8u * (txy >> 16) + (slot >> 3);
    re.q = (slot < 64u && px < width && py < height) ? lt * 64u + slot : ~0u;
    re.s[0] = re.s[1] = re.s[2] = 0.0;
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

// The viewport point's two terms, each one fixed sequence of fp32 operations: shader.comp:43's
// pixel corner pixel00 + x delta_u + y delta_v, and :48-49's jitter in world units
// jx delta_u + jy delta_v (TraceParams.jitter); the sample's point is their sum.
__device__ __forceinline__ f3 viewport_corner(f3 p00, f3 du, f3 dv, uint32_t x, uint32_t y) {
    return add(add(p00, scale((float)x, du)), scale((float)y, dv));
}

__device__ __forceinline__ f3 viewport_jitter(f3 du, f3 dv, float2 jt) {
    return add(scale(jt.x, du), scale(jt.y, dv));
}

// The jitter term of sample i and a hit sphere's shading rows, from the LDS copy the SMEM scan
// stages for small scenes (TraceParams.stage_*), else from global memory.
template <bool kStageable>
__device__ __forceinline__ float4 jitter_at(const TraceParams& p, const float4* lds, int i) {
    if constexpr (kStageable) {
        if (p.stage_spp != 0u) return lds[3u * p.stage_spheres + (uint32_t)i];
    }
    return p.jitter[i];
}

template <bool kStageable>
__device__ __forceinline__ void shading_rows(const TraceParams& p, const float4* lds, int best,
                                             float4& cr, float4& sh, float4& mat) {
    if constexpr (kStageable) {
        if (p.stage_spp != 0u) {
            const uint32_t ns = p.stage_spheres;
            cr = lds[best];
            sh = lds[ns + best];
            mat = lds[2u * ns + best];
            return;
        }
    }
    cr = p.center_radius[best];
    sh = p.shade[best];
    mat = p.material[best];
}

// kCull: 0 = linear scan (kLds: table in LDS), 1 = culled scan, 2 = per-lane culled scan
// with the group tables copied to LDS, 3 = per-lane culled scan on global tables.
template <bool kLds, bool kStats, int kCull = 0, bool kCostOrder = false>
__device__ __forceinline__ void trace_impl(const TraceParams& p_arg, float4* lds_dyn) {
    // P: the kernel arguments, read through a pointer to the kernarg segment (the kernels' only
    // argument) that the persistent loop makes opaque at the top of every iteration (below), so
    // that the compiler re-reads the arguments it needs (scalar loads from the constant cache)
    // instead of keeping every value derived from them live across the loop. That freed the ~75
    // SGPRs the flat kernel spilled to VGPR lanes (a v_readlane per reload): C4 +2.6%, stress
    // scene +5%, same bits.
    (void)p_arg;
    const TraceParams* pargs = reinterpret_cast<const TraceParams*>(
        (__attribute__((address_space(4))) const TraceParams*)__builtin_amdgcn_kernarg_segment_ptr());
#define P (*pargs)
    const int n = P.nspheres;
    float4* const lds_geom = lds_dyn;
    if constexpr (kLds) {
        const int nq = 4 * (((n + 3) >> 2) + 1);
        for (int i = threadIdx.x; i < nq; i += blockDim.x) lds_geom[i] = P.geom[i];
        __syncthreads();
    }
    // The SMEM scan of a small scene reads the shading rows and the jitter from an LDS copy
    // (TraceParams.stage_*: [stage_spheres] center_radius, shade, material, then the jitter).
    constexpr bool kStageable = kCull == 0 && !kLds;
    if constexpr (kStageable) {
        if (P.stage_spp != 0u) {
            const uint32_t ns = P.stage_spheres;
            for (uint32_t i = threadIdx.x; i < ns; i += blockDim.x) {
                lds_dyn[i] = P.center_radius[i];
                lds_dyn[ns + i] = P.shade[i];
                lds_dyn[2u * ns + i] = P.material[i];
            }
            for (uint32_t i = threadIdx.x; i < P.stage_spp; i += blockDim.x)
                lds_dyn[3u * ns + i] = P.jitter[i];
            __syncthreads();
        }
    }

    // group-pair boxes: the flat scan reads the near/far layout (80 B per pair), the others
    // the pair-SoA one (64 B)
    constexpr bool kFlat = kCull == 4 || kCull == 5 || kCull == 6;
    const float4* tbound = kFlat ? P.cbound_nf : P.cbound;
    const float4* tnode = P.cnode_nf;              // the flat scans' chunk passes
    const float4* tgroup = P.cgroup + 5 * P.nbig;  // the hierarchy's group records
    // the flat scan's stacks: after the LDS tables (kCull 4: all tables; kCull 6: the boxes,
    // with the group records in global memory), or alone with the tables in global memory and
    // 32-bit entries (kCull 5)
    constexpr int kFmt = kCull == 5 ? 2 : kCull == 6 ? 1 : 0;  // stack entry format
    constexpr bool kGRec = kCull == 5 || kCull == 6;
    constexpr bool kChunks = kCull == 5 || kCull == 6;
    // float4s per node record of the near/far box tables (a node's 8 group boxes, a chunk's 8
    // node boxes: 4 pairs x 80 B): in LDS padded by 16 B, so that the records of nodes n and
    // n + 2 no longer start on the same LDS bank (stride 84 dwords instead of 80: eight start
    // banks for the ds_read2_b64 of a 16-lane group instead of two)
    constexpr uint32_t kNS = (kCull == 4 || kCull == 6) ? 21u : 20u;
    // the flat scans' per-wave stacks (the LDS-table kernel has no chunk level)
    using WS = WaveScratch<kFmt, kChunks>;
    WS* ws = nullptr;
    GroupTab<kGRec> tg{tgroup};  // the flat scans' view of the group records
    if constexpr (kCull == 2) {
        const int nb = (P.ncgroups >> 1) * 4, ng = P.ncgroups * 5;
        for (int i = threadIdx.x; i < nb; i += blockDim.x) lds_geom[i] = tbound[i];
        for (int i = threadIdx.x; i < ng; i += blockDim.x) lds_geom[nb + i] = tgroup[i];
        __syncthreads();
        tbound = lds_geom;
        tgroup = lds_geom + nb;
    }
    if constexpr (kCull == 4) {  // LDS: near/far boxes, 80-B group records with uint16 indices
        const int nb = (P.ncgroups >> 3) * kNS, ng = P.ncgroups * 5;
        {  // and the chunks' node boxes (near/far, padded records) after the group records
            const int nn = ((P.ncgroups + 63) >> 6) * kNS;
            for (int i = threadIdx.x; i < nn; i += blockDim.x)
                if (i % kNS != 20u) lds_geom[nb + ng + i] = tnode[i - i / kNS];
        }
        for (int i = threadIdx.x; i < nb; i += blockDim.x)
            if (i % kNS != 20u) lds_geom[i] = tbound[i - i / kNS];
        for (int i = threadIdx.x; i < ng; i += blockDim.x) {
            float4 v = tgroup[i];
            if (i % 5 == 4) {  // member indices < 2^16 (<= 1024 groups), as uint16 (-1: 0xffff)
                const uint32_t lo = ((uint32_t)__float_as_int(v.x) & 0xffffu) |
                                    ((uint32_t)__float_as_int(v.y) << 16);
                const uint32_t hi = ((uint32_t)__float_as_int(v.z) & 0xffffu) |
                                    ((uint32_t)__float_as_int(v.w) << 16);
                v = make_float4(__uint_as_float(lo), __uint_as_float(hi), 0.0f, 0.0f);
            }
            lds_geom[nb + i] = v;
        }
        __syncthreads();
        tbound = lds_geom;
        tg.geom = lds_geom + nb;
        tnode = lds_geom + nb + ng;
        ws = reinterpret_cast<WS*>(lds_geom + nb + ng + ((P.ncgroups + 63) >> 6) * kNS) +
             (threadIdx.x >> 6);
        static_assert(kNS == 21u && sizeof(WS) == kWaveScratchBytes8,
                      "host LDS size (capi.cpp select_kernel)");
    }
    if constexpr (kCull == 5) ws = reinterpret_cast<WS*>(lds_geom) + (threadIdx.x >> 6);
    if constexpr (kCull == 6) {  // LDS: near/far group boxes, near/far node boxes (whole chunks)
        const int nb = (P.ncgroups >> 3) * kNS, nn = ((P.ncgroups + 63) >> 6) * kNS;
        for (int i = threadIdx.x; i < nb; i += blockDim.x)
            if (i % kNS != 20u) lds_geom[i] = tbound[i - i / kNS];
        for (int i = threadIdx.x; i < nn; i += blockDim.x)
            if (i % kNS != 20u) lds_geom[nb + i] = tnode[i - i / kNS];
        __syncthreads();
        tbound = lds_geom;
        tnode = lds_geom + nb;
        ws = reinterpret_cast<WS*>(lds_geom + nb + nn) +
             (threadIdx.x >> 6);
    }
    const uint32_t lane = threadIdx.x & 63u;
    // stats builds: this wave's row of region counters (null in the product: calls fold away)
    uint32_t* rrow = nullptr;
    if constexpr (kStats) {
        if (P.region)
            rrow = P.region + (blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)) * kRegions;
    }
    const f3 p00 = mk(P.cam[0], P.cam[1], P.cam[2]);
    const f3 du = mk(P.cam[3], P.cam[4], P.cam[5]);
    const f3 dv = mk(P.cam[6], P.cam[7], P.cam[8]);
    const f3 cam = mk(P.cam[9], P.cam[10], P.cam[11]);
    const uint32_t nchunks = (uint32_t)P.nchunks;
    const bool reverse = (P.flags & kFlagReverseOrder) != 0;
    const bool chunk_minor = (P.flags & kFlagChunkMinor) != 0;

    bool done = false, need = true;
    bool newray = false;  // the lane's next sample's camera ray is set up at the next fetch
    bool fin = false;  // the lane's quantum is finished and its sum in acc not yet added
    bool fresh = false;  // the lane's ray is a camera ray not yet traced (flat scan)
    // flat scan: a main-scan hit waits for the next iteration's shading (pend_t, pend_best;
    // pend_best < 0: none), which it shares with that iteration's camera rays
    float pend_t = 0.0f;
    int pend_best = -1;  // -1: none; kPendSky: a sky segment
    int sample = 0, sample_end = 0, pass = 0;
    uint32_t q = 0;
    uint32_t pxy = 0;  // the item's pixel: y << 16 | x
    f3 o = mk(0.f, 0.f, 0.f), d = o, atten = o, acc = o;
    // shader.comp:43-52: the camera ray of sample s of the lane's pixel, (corner + jitter) - center,
    // both terms from tables built with the same operations (TraceParams.jitter per sample index,
    // TraceParams.corner per local slot) instead of 25 VALU instructions at every sample start:
    // C4 +1.1%, C3 +1.1% (profiles/r04_ab_log.md). The linear scans (C2: a small, latency-bound
    // frame, -6% with the corner's load) recompute the corner from pxy.
    auto camera_dir = [&](int s) {
        f3 c;
        if constexpr (kCull != 0) {  // the culled scans: the corner from its table
            const float4 c4 = P.corner[q & kQMask];
            c = mk(c4.x, c4.y, c4.z);
        } else {  // the linear scans (small, latency-bound frames): computed, no load
            c = viewport_corner(p00, du, dv, pxy & 0xffffu, pxy >> 16);
        }
        const float4 j = jitter_at<kStageable>(P, lds_dyn, s);
        return sub(add(c, mk(j.x, j.y, j.z)), cam);
    };
    uint32_t segs = 0;  // this lane's segments (< 2^32: ~2.4e5 per lane at the C5 workload)
    uint64_t st_iters = 0, st_active = 0, st_hitgroups = 0, st_fetch = 0;
    // issued work (tally): half-groups (sphere-pair tests of the camera lists count one, group
    // tests two) and box tests
    uint32_t w_halves = 0, w_bounds = 0;
    PhaseTicks pt;                         // stats builds: wave clock per phase
    uint64_t t_begin = 0;
    if constexpr (kStats) t_begin = ticks();
#ifdef VCRT_WAVE_END_TIMES
    const unsigned long long t_start_rt = __builtin_amdgcn_s_memrealtime();
    unsigned long long t_drained_rt = ~0ull;
#endif
    // the wave's current block of items (wave-uniform); 64 = exhausted, fetch a new one
    const uint32_t total_blocks = P.total_items >> 6;
    uint32_t blk_next = 64u, blk_lt = 0u, blk_chunk = 0u, blk_tx = 0u, blk_ty = 0u;
    uint32_t q_x = blockIdx.x & (kQueues - 1u), q_drained = 0u;  // the wave's queue; found empty
    uint32_t blk_nch = nchunks;  // chunks per pixel of the block's part (head or tail)
    uint32_t fetch_waited = 0u;  // wave-iterations the fetch was deferred (flat scans)
    bool blk_tail = false;
    // the wave's accumulation ring (see RingEntry): next entry to hand out; the current block's
    // first pixel slot and first entry + 1 (0: the block's items add to global memory)
    RingEntry* const ring =
        P.ring_n ? reinterpret_cast<RingEntry*>(reinterpret_cast<char*>(lds_dyn) + P.ring_off) +
                       __builtin_amdgcn_readfirstlane(threadIdx.x >> 6) * P.ring_n
                 : nullptr;
    uint32_t ring_pos = 0u, blk_ps0 = 0u, blk_ring = 0u;
    if (ring) {
        for (uint32_t i = lane; i < P.ring_n; i += 64u) ring[i].q = ~0u;
        __builtin_amdgcn_wave_barrier();
    }
    if constexpr (kFlat) {
        if (lane < 2u) ws->work[lane] = 0u;
        __builtin_amdgcn_wave_barrier();
    }

    // Shades a traced segment (textures.glsl, or the sky of functions.glsl:85-89) and advances
    // the lane's path: accumulate and start the next sample's camera ray (returns true), or
    // finish the chunk (need), or continue with the bounced ray.
    // defer_ray: a sample that ends here leaves its next camera ray to the next iteration's fetch
    // (which sets up new items' first rays anyway; used after the main scan, whose lanes trace
    // that ray no earlier than the next camera fast trace)
    auto shade_and_advance = [&](float max_t, int best, bool defer_ray, uint32_t rb) -> bool {
        bool ended = false, fresh_cam = false;
        f3 contrib = mk(0.f, 0.f, 0.f);
        region(rrow, rb + reg::kShEntry);
        if (best >= 0) {
            region(rrow, rb + reg::kShHit);
            float4 cr, sh, mat;
            shading_rows<kStageable>(P, lds_dyn, best, cr, sh, mat);
            const f3 point = add(scale(max_t, d), o);
            // normal = (point - centre) / radius: the unscaled division with one reciprocal
            // (exact: candidate_t_fast's argument) for numerators and radius in [2^-40, 2^30]
            // (the radius by a host flag), else hipcc's full division in a real branch
            const f3 pcv = sub(point, mk(cr.x, cr.y, cr.z));
            const float yr = recip_a(cr.w);
            f3 normal = mk(div_a(pcv.x, cr.w, yr), div_a(pcv.y, cr.w, yr), div_a(pcv.z, cr.w, yr));
            const float nmin = fminf(fminf(fabsf(pcv.x), fabsf(pcv.y)), fabsf(pcv.z));
            const float nmax = fmaxf(fmaxf(fabsf(pcv.x), fabsf(pcv.y)), fabsf(pcv.z));
            if (!((P.flags & kFlagRadiiSafe) != 0u && nmin >= 0x1p-40f && nmax <= 0x1p30f)) {
                asm volatile("");
                region(rrow, rb + reg::kShNormalDiv);
                normal = divs(pcv, cr.w);
            }
            const int type = (int)mat.x;
            const f3 albedo = mk(sh.x, sh.y, sh.z);
            const float param = sh.w;
            // rand(dir.xy), rand(dir.xz), rand(dir.yz) for lambertian/metal (functions.glsl:43),
            // rand(point.xy) for glass (textures.glsl:51): three sines for every hit lane
            float s1, s2, s3;
            bool sin_fb = false;
            sin3<true>((type == 3) ? rand_arg(point.x, point.y) : rand_arg(d.x, d.y),
                       rand_arg(d.x, d.z), rand_arg(d.y, d.z), s1, s2, s3,
                       (cdouble*)&P.sin_c[0], kStats ? &sin_fb : nullptr);
            if constexpr (kStats) {
                if (__ballot(sin_fb)) region(rrow, rb + reg::kShSinFallback);
            }
            const float r1 = rand_of_sin(s1);
            if (type == 1 || type == 2) {
                region(rrow, rb + reg::kShLamMetal);
                const float r2 = rand_of_sin(s2);
                const float r3 = rand_of_sin(s3);
                const f3 ru = mk(r1, r2, r3);  // random_in_unit_sphere(dir): normalize
                const f3 u = divs(ru, sqrt_fast(dot(ru, ru), rrow));
                if (type == 1) {
                    region(rrow, rb + reg::kShLam);
                    d = add(normal, u);
                    atten = scale(param, mul(atten, albedo));
                } else {
                    region(rrow, rb + reg::kShMetal);
                    d = add(reflect(d, normal), scale(param, u));
                    atten = mul(atten, albedo);
                }
                o = point;
            } else if (type == 3) {
                region(rrow, rb + reg::kShGlass);
                const f3 reflected = reflect(d, normal);
                f3 outward;
                float ni, cosine;
                const float dn = dot(d, normal);
                if (dn > 0.0f) {
                    region(rrow, rb + reg::kShGlassIn);
                    outward = neg(normal);
                    ni = param;
                    cosine = sqrt_fast(1.0f - param * param * (1.0f - dn * dn), rrow);
                } else {
                    region(rrow, rb + reg::kShGlassOut);
                    outward = normal;
                    ni = mat.y;  // 1.0f / param
                    cosine = -dn;
                }
                f3 refracted = mk(0.f, 0.f, 0.f);
                float reflect_prob = 1.0f;
                const float dt = dot(d, outward);
                const float disc = 1.0f - ni * ni * (1.0f - dt * dt);
                if (disc > 0.0f) {
                    region(rrow, rb + reg::kShGlassRefract);
                    const float sd = sqrt_fast(disc, rrow);
                    refracted = sub(scale(ni, sub(d, scale(dt, outward))), scale(sd, outward));
                    reflect_prob = schlick_r0(cosine, mat.z);  // schlick(cosine, param)
                }
                o = point;
                d = (r1 < reflect_prob) ? reflected : refracted;
            }
            ++pass;
            if (pass >= P.max_depth) ended = true;  // undefined GLSL return -> vec3(0)
        } else {
            region(rrow, rb + reg::kShSky);
            const float len = sqrt_fast(dot(d, d), rrow);  // length(d)
            contrib = mul(atten, sky_factor(d.y / len));
            ended = true;
        }

        if (ended) {
            region(rrow, rb + reg::kShEnded);
            acc = add(acc, contrib);  // the quantum's fp32 sum in sample order
            ++sample;
            if (sample == sample_end) {
                region(rrow, rb + reg::kShItemEnd);
                // the item is done: its last quantum's sum in acc is retired at the top of the
                // next iteration (few registers are live there: the accumulation code stays out
                // of shading)
                fin = true;
                need = true;
            } else {
                // a quantum of G samples ends inside the item: its sum is retired the same way,
                // and the item goes on with its next sample
                if (((uint32_t)sample & P.quantum_mask) == 0u) fin = true;
                if (defer_ray) {
                    newray = true;
                } else {
                    region(rrow, rb + reg::kShNewRay);
                    d = camera_dir(sample);
                    o = cam;
                    atten = mk(1.f, 1.f, 1.f);
                    pass = 0;
                    fresh_cam = true;
                }
            }
        }
        return fresh_cam;
    };

    for (;;) {
        {  // the argument pointer, opaque to the optimiser (an asm result) and wave-uniform
           // (readfirstlane: loads through it stay scalar), in the constant address space
            uint64_t a = reinterpret_cast<uint64_t>(pargs);
            asm volatile("" : "+s"(a));
            const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a);
            const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
            pargs = reinterpret_cast<const TraceParams*>(
                (__attribute__((address_space(4))) const TraceParams*)(((uint64_t)hi << 32) | lo));
        }
        region(rrow, reg::kIter);
        uint64_t t_top = 0;
        if constexpr (kStats) {
            t_top = ticks();
            const uint64_t fm = __ballot(fin);
            pt.retire_iters += fm != 0u;
            pt.quanta += (uint64_t)__popcll(fm);
        }
        if (fin) {  // ---- retire the finished quantum: its sum to the pixel ----
            region(rrow, reg::kRetire);
            fin = false;
            if constexpr (!kFlat || kCostOrder) {  // the item's segments (the cost order)
                if (P.pixel_cost != nullptr && need) atomicAdd(P.pixel_cost + (q & kQMask), segs);
            }
            if ((P.flags & kFlagDirect) != 0u) {
                // the pixel's one chunk: color /= SPP in fp32 (shader.comp:56)
                const uint32_t out_index =
                    P.world == 1 ? (pxy >> 16) * (uint32_t)P.width + (pxy & 0xffffu) : q & kQMask;
                P.out[out_index] = make_float4(acc.x / P.spp_total, acc.y / P.spp_total,
                                               acc.z / P.spp_total, 1.0f);
            } else {
                // the quantum sum, quantized: RN_even(S * 2^s) (an integer below 2^44), summed
                // exactly over the pixel's quanta in double (vcrt_math.h "Accumulation"). The
                // scale: 2^32 from s + 128 in the flags' top byte (scalar ops, no load), or with
                // kFlagPixelScale the pixel's own from pixel_emax (a wave-uniform branch).
                // (Three compares with |.| modifiers: NaN compares false; the rare cases in a
                // real branch, so the common path converts without selects.)
                float sc = __uint_as_float(
                    ((P.flags >> kFlagScaleShift) + (127u - (uint32_t)kFlagScaleBias)) << 23);
                const uint32_t qi = q & kQMask, ent = q >> kRingQBits;
                if ((P.flags & kFlagPixelScale) != 0u) {
                    asm volatile("");
                    sc = __uint_as_float((uint32_t)(pixel_scale_log2(P.pixel_emax[qi]) + 127) << 23);
                }
                float ax = acc.x * sc, ay = acc.y * sc, az = acc.z * sc;
                if (!(fabsf(ax) < kAccumQLimit && fabsf(ay) < kAccumQLimit &&
                      fabsf(az) < kAccumQLimit)) {
                    asm volatile("");
                    region(rrow, reg::kRetireNan);
                    if (__builtin_isfinite(acc.x) && __builtin_isfinite(acc.y) &&
                        __builtin_isfinite(acc.z)) {
                        // an outlier quantum: its pixel needs a smaller scale; the host renders
                        // the frame again with pixel_emax (this frame's sums are discarded)
                        const uint32_t mb = __float_as_uint(
                            fmaxf(fabsf(acc.x), fmaxf(fabsf(acc.y), fabsf(acc.z))));
                        atomicMax(P.pixel_emax + qi, mb);
                        atomicMax(P.outlier_max, mb);
                    }
                    ax = ay = az = __builtin_nanf("");  // infinite or NaN radiance: a NaN pixel
                }
                const double v0 = (double)__builtin_rintf(ax);
                const double v1 = (double)__builtin_rintf(ay);
                const double v2 = (double)__builtin_rintf(az);
                // the pixel's ring entry while it still holds this pixel (LDS atomics; a claim
                // that takes the entry for another pixel clears the lane's entry field), else
                // global memory (two branches: a pointer that may be either would make flat
                // atomics, whose completion every later LDS wait would wait for)
#ifdef VCRT_KO_RETIRE_ADD  // timing knock-out (wrong image): the quanta computed, not added
                constexpr bool kAdd = false;
                asm volatile("" ::"v"(v0), "v"(v1), "v"(v2), "v"(qi), "v"(ent));
#else
                constexpr bool kAdd = true;
#endif
                if (kAdd && ent != 0u) {
                    region(rrow, reg::kRetireRing);
                    double* s = ring[ent - 1u].s;
                    atomicAdd(s + 0, v0);
                    atomicAdd(s + 1, v1);
                    atomicAdd(s + 2, v2);
                } else if (kAdd) {
                    region(rrow, reg::kRetireGlobal);
                    double* s = P.accum + 4u * qi;
                    atomicAdd(s + 0, v0);
                    atomicAdd(s + 1, v1);
                    atomicAdd(s + 2, v2);
                }
            }
            acc = mk(0.f, 0.f, 0.f);  // the next quantum (of this item or the next) sums from 0
        }
        if (newray) {  // the next sample's camera ray (shader.comp:48-52), deferred by the sky
            region(rrow, reg::kNewRay);
            newray = false;
            d = camera_dir(sample);
            o = cam;
            atten = mk(1.f, 1.f, 1.f);
            pass = 0;
            fresh = true;
        }
        // ---- lanes whose item is finished take the next slots of the wave's current block
        //      (one tile x chunk = 64 items); a new block costs one atomic per wave ----
        uint64_t t_fetch = 0;
        if constexpr (kStats) {
            t_fetch = ticks();
            pt.retire += t_fetch - t_top;
        }
        // The loop only hands out slots; the lane state is set up once after it (setting it up
        // inside made the compiler copy ~20 live registers around the loop on every pass).
        bool got = false;
        uint32_t g_lt = 0u, g_chunk = 0u, g_slot = 0u, g_px = 0u, g_py = 0u, g_ent = 0u;
        int g_s0 = -1, g_s1 = 0;  // a stolen sample range (the drain below), else -1
        uint64_t need_mask = __ballot(need && !done);
        if constexpr (kFlat) {
            // deferred fetches (TraceParams.fetch_min / fetch_wait): while fewer than fetch_min
            // lanes need an item and other lanes still have work, the wave skips the fetch for up
            // to fetch_wait iterations (the waiting lanes idle; the fetch runs for more at once)
            if (need_mask != 0u) {
                if ((uint32_t)__popcll(need_mask) < P.fetch_min && fetch_waited < P.fetch_wait &&
                    __ballot(!need && !done) != 0u) {
                    ++fetch_waited;
                    need_mask = 0u;
                } else {
                    fetch_waited = 0u;
                }
            }
        }
        if constexpr (kStats) pt.fetch_iters += need_mask != 0u;
        while (need_mask) {
            region(rrow, reg::kFetchTrip);
            if (blk_next >= 64u) {
                if constexpr (kStats && kCull == 0) ++st_fetch;
                // kQueues queues, each on workgroups of one XCD (workgroups are dispatched to
                // the XCDs round robin): queue x hands out blocks kQueues k + x on its own
                // counter; a wave whose queue is drained moves on to the next open one, and is
                // done when it has found every queue drained
                uint32_t b = ~0u;
                while (b == ~0u && q_drained < kQueues) {
                    const int leader = __ffsll((unsigned long long)__ballot(1)) - 1;
                    const uint32_t nq = (total_blocks + kQueues - 1u - q_x) / kQueues;
                    uint32_t k = 0;
                    const uint32_t amt = 1u;
                    if ((int)lane == leader) k = atomicAdd(P.work + kQueueStride * q_x, amt);
                    k = __builtin_amdgcn_readfirstlane(__shfl(k, leader));
                    if (k < nq) {
                        b = kQueues * k + q_x;
                        break;
                    }
#ifdef VCRT_OLD_DRAIN
                    ++q_drained;
                    q_x = (q_x + 1u) & (kQueues - 1u);
#else
                    // this queue is drained: read every queue's counter at once (one load per
                    // lane; a counter only grows, so "drained" read here is final) and move to
                    // the next open queue after q_x, or finish when none is open. (Trying the
                    // queues one atomic at a time made every wave of the grid issue kQueues
                    // serialized atomics on the same kQueues counters at the end of a frame:
                    // ~0.25 ms of tail per launch.)
                    const uint64_t act = __ballot(1);
                    const uint32_t na = (uint32_t)__popcll(act), rk = lanes_below(act);
                    uint32_t best = 0u;  // kQueues - (distance of the nearest open queue)
                    for (uint32_t base = 0; base < kQueues; base += na) {
                        const uint32_t dq = base + rk + 1u;  // distance from q_x: 1 .. kQueues
                        uint32_t v = 0u;
                        if (dq <= kQueues) {
                            const uint32_t qq = (q_x + dq) & (kQueues - 1u);
                            const uint32_t cnt = __hip_atomic_load(P.work + kQueueStride * qq,
                                                                   __ATOMIC_RELAXED,
                                                                   __HIP_MEMORY_SCOPE_AGENT);
                            const uint32_t nqq = (total_blocks + kQueues - 1u - qq) / kQueues;
                            if (cnt < nqq) v = kQueues + 1u - dq;
                        }
                        best = max(best, wave_max_small<6>(v));
                    }
                    // (each failed atomic is on a queue that then reads drained: at most
                    // kQueues of them per wave, as before)
                    ++q_drained;
                    if (best == 0u) {
                        q_drained = kQueues;
                    } else {
                        q_x = (q_x + (kQueues + 1u - best)) & (kQueues - 1u);
                    }
#endif
                }
                if (b == ~0u) {  // queues drained: lanes still wanting work are done
#ifdef VCRT_WAVE_END_TIMES
                    if (t_drained_rt == ~0ull) t_drained_rt = __builtin_amdgcn_s_memrealtime();
#endif
                    if (need) done = true;
                    break;
                }
                if constexpr (kStats) ++pt.blk_fetches;
                region(rrow, reg::kBlock);
                // block b = (local tile lt, chunk) of the head, then of the tail: wave-uniform
                // tile origin and sample range; reversed within each part
                if constexpr (!kFlat || kCostOrder) {  // cost order (any part; a scalar load)
                    if (P.block_order != nullptr)
                        b = ((__attribute__((address_space(4))) const uint32_t*)P.block_order)[b];
                }
                blk_tail = b >= P.blocks_head;
                if (blk_tail) b -= P.blocks_head;
                if (reverse) b = (blk_tail ? total_blocks - P.blocks_head : P.blocks_head) - 1u - b;
                blk_nch = blk_tail ? (uint32_t)P.tail_nchunks : nchunks;
                blk_lt = b / blk_nch;
                blk_chunk = b - blk_lt * blk_nch;
                tile_of(blk_lt, (uint32_t)P.rank, (uint32_t)P.world, P.tiles_x, &blk_tx, &blk_ty);
                blk_next = 0u;
                // ring entries for the block's pixel slots ps0 .. ps1 (chunk-minor items
                // 64 c .. 64 c + 63 of the tile are (i / nch, i % nch)): flushed and set up by
                // one lane each (the loop top runs with every lane of the wave)
                blk_ring = 0u;
                if (ring && chunk_minor && __builtin_amdgcn_read_exec() == ~0ull) {
                    const uint32_t ps0 = (64u * blk_chunk) / blk_nch;
                    const uint32_t np = (64u * blk_chunk + 63u) / blk_nch - ps0 + 1u;
                    if (np <= P.ring_n) {
                        region(rrow, reg::kBlockRing);
                        if (lane < np)
                            ring_claim(ring, ring_pos + lane, P.ring_n, P.accum, ps0 + lane,
                                       blk_lt, (blk_ty << 16) | blk_tx, (uint32_t)P.width,
                                       (uint32_t)P.height);
                        __builtin_amdgcn_wave_barrier();
                        // a lane whose item's entry is among those just claimed (its own, or
                        // the one of an item handed to it earlier in this fetch) loses it: the
                        // item's later quanta go to global memory
                        const uint32_t rn = P.ring_n, pos = ring_pos;
                        auto keep = [rn, pos, np](uint32_t ent) {
                            uint32_t rel = ent + rn - 1u - pos;
                            if (rel >= rn) rel -= rn;
                            return (ent != 0u && rel < np) ? 0u : ent;
                        };
                        q = (q & kQMask) | (keep(q >> kRingQBits) << kRingQBits);
                        g_ent = keep(g_ent);
                        blk_ps0 = ps0;
                        blk_ring = ring_pos + 1u;
                        ring_pos += np;
                        if (ring_pos >= P.ring_n) ring_pos -= P.ring_n;
                    }
                }
            }
            const uint32_t avail = 64u - blk_next;
            const uint32_t mine = lanes_below(need_mask);
            if (need && !done && mine < avail) {
                uint32_t slot = blk_next + mine, ch = blk_chunk;
                if (chunk_minor) {  // item 64 j + slot of the tile = (pixel, chunk), chunk-minor
                    // i / n by the host's magic multiplier (exact for every i < 64 n, checked
                    // by the host; 0: none): C4 8-way shards -1% against hipcc's division
#ifdef VCRT_NO_MAGIC
                    const uint32_t m = 0u;
#else
                    const uint32_t m = blk_tail ? P.nch_magic[1] : P.nch_magic[0];
#endif
                    const uint32_t i = 64u * blk_chunk + slot;
                    if (m != 0u) {
                        slot = __umulhi(i, m);
                    } else {
                        asm volatile("");
                        slot = i / blk_nch;
                    }
                    ch = i - slot * blk_nch;
                }
                if (blk_tail) ch |= 0x10000u;  // chunk ch of the tail
                const uint32_t px = 8u * blk_tx + (slot & 7u), py = 8u * blk_ty + (slot >> 3);
                if (px < (uint32_t)P.width && py < (uint32_t)P.height) {  // edge tiles: skip
                    got = true;
                    g_lt = blk_lt;
                    g_chunk = ch;
                    g_slot = slot;
                    g_px = px;
                    g_py = py;
                    need = false;
                    g_ent = 0u;
                    if (blk_ring) {  // the pixel's ring entry (+ 1)
                        uint32_t ei = blk_ring + (slot - blk_ps0);
                        if (ei > P.ring_n) ei -= P.ring_n;
                        g_ent = ei;
                    }
                }
            }
            blk_next += min((uint32_t)__popcll(need_mask), avail);
            need_mask = __ballot(need && !done);
        }
#ifndef VCRT_NO_STEAL
        // ---- the drain: once every queue is empty, an idle lane takes the later quanta of
        //      the wave's longest remaining item (the victim keeps the quantum in progress and
        //      half of the rest). Quanta are summed on their own and added exactly, so any lane
        //      may trace any whole quantum of a pixel: the same bits, the same segments. ----
        if (q_drained >= kQueues && (P.flags & kFlagDirect) == 0u) {
            uint64_t idle = __ballot(done);
            if (idle != 0u) {
                const int gm = (int)P.quantum_mask, G = gm + 1;
                uint32_t rem = 0u;  // whole quanta after the one in progress
                if (!done && !need) {
                    const int next = (sample & ~gm) + G;
                    if (sample_end > next) rem = (uint32_t)((sample_end - next + gm) / G);
                }
                while (idle != 0u) {
                    region(rrow, reg::kSteal);
                    const uint32_t top = wave_max_small<10>(rem);  // <= kAccumMaxChunks
                    if (top == 0u) break;
                    const uint32_t victim = (uint32_t)__builtin_ctzll(__ballot(rem == top));
                    const uint32_t thief = (uint32_t)__builtin_ctzll(idle);
                    idle &= idle - 1u;
                    const uint32_t give = (top + 1u) >> 1;
                    const int v_sample = __builtin_amdgcn_readlane(sample, victim);
                    const int v_end = __builtin_amdgcn_readlane(sample_end, victim);
                    const uint32_t v_q = __builtin_amdgcn_readlane(q, victim);
                    const uint32_t v_pxy = __builtin_amdgcn_readlane(pxy, victim);
                    const int cut = (v_sample & ~gm) + G * (int)(1u + top - give);
                    if (lane == victim) {
                        sample_end = cut;
                        rem = top - give;
                    }
                    if (lane == thief) {
                        got = true;
                        done = false;
                        need = false;
                        g_lt = (v_q & kQMask) >> 6;
                        g_slot = v_q & 63u;
                        g_ent = v_q >> kRingQBits;
                        g_px = v_pxy & 0xffffu;
                        g_py = v_pxy >> 16;
                        g_s0 = cut;
                        g_s1 = v_end;
                        // no victim before its range is set up (the got block below): its
                        // sample / sample_end / q still name the item it finished
                        rem = 0u;
                    }
                }
            }
        }
#endif
        if constexpr (kStats) pt.items_cur += (uint64_t)__popcll(__ballot(got));
        if (got) {
            region(rrow, reg::kItem);
            q = (g_lt * 64u + g_slot) | (g_ent << kRingQBits);
            pxy = (g_py << 16) | g_px;
            if constexpr (!kFlat || kCostOrder) {
                if (P.pixel_cost != nullptr) atomicSub(P.pixel_cost + g_lt * 64u + g_slot, segs);
            }
            // the item's samples: the four partition values are wave-uniform, read by scalar
            // loads and selected per lane (left to itself the compiler selected their kernarg
            // addresses per lane and read them with vector loads, whose latency the jitter
            // load's address then waited for: two dependent memory round trips per fetch)
            const bool tail = g_chunk >= 0x10000u;
#ifdef VCRT_NO_SCALAR_PART
            const int k_head = P.chunk, k_tail = P.tail_chunk, t_start = P.tail_start,
                      n_spp = P.spp;
#else
            const int k_head = __builtin_amdgcn_readfirstlane(P.chunk);
            const int k_tail = __builtin_amdgcn_readfirstlane(P.tail_chunk);
            const int t_start = __builtin_amdgcn_readfirstlane(P.tail_start);
            const int n_spp = __builtin_amdgcn_readfirstlane(P.spp);
#endif
            const int k = tail ? k_tail : k_head;
            sample = (tail ? t_start : 0) + (int)(g_chunk & 0xffffu) * k;
            sample_end = min(sample + k, tail ? n_spp : t_start);
#ifndef VCRT_NO_STEAL
            if (g_s0 >= 0 && g_s0 < g_s1) {  // a stolen range of whole quanta (never empty)
                sample = g_s0;
                sample_end = g_s1;
            }
#endif
            // first camera ray of the chunk, shader.comp:48-52
            d = camera_dir(sample);
            o = cam;
            atten = mk(1.f, 1.f, 1.f);
            pass = 0;
            fresh = true;
        }
        if constexpr (kStats) pt.fetch += ticks() - t_fetch;
        const uint64_t live = __ballot(!done);
        if (live == 0) break;
        if constexpr (kStats) {
            ++st_iters;
            st_active += (uint64_t)__popcll(live);
        }
        if (done) continue;

        // ---- flat scan: a camera ray not yet traced (started by the last shading or by the
        //      fetch) is traced first, from its pixel quarter's group list (the big list, then
        //      the listed groups, per lane, with hit_sphere's consider rule: the same sphere
        //      and t as the flat scan), and shaded; the lane then takes its first bounce
        //      through this iteration's scan. The per-wave costs of an iteration (uniform
        //      levels, ray setup, block fetch) are so shared by two segments of such lanes. ----
        if constexpr (kFlat) {
            uint64_t t_cam = 0;
            if constexpr (kStats) t_cam = ticks();
            uint32_t inf = 15u;
            if (fresh && P.prim_info != nullptr)  // the sphere list of the item's 4x4 quarter
                inf = P.prim_info[2u * (((q & kQMask) >> 6) * 4u + (((q >> 5) & 1u) << 1) +
                                        ((q >> 2) & 1u)) +
                                  1u];
            const float aa = dot(d, d);
            const bool cam_now = fresh && (inf & 15u) != 15u && (P.flags & kFlagSceneBounded) != 0 &&
                                 aa >= 0x1p-20f && aa <= 0x1p60f && fabsf(o.x) <= 0x1p30f &&
                                 fabsf(o.y) <= 0x1p30f && fabsf(o.z) <= 0x1p30f;
            float mt = __uint_as_float(vconst<0x47c35000u>());  // kInfinity
            int bst = (int)vconst<0xffffffffu>();                // -1
            if (__ballot(cam_now)) {
                region(rrow, reg::kCam);
                if constexpr (kStats) {
                    ++pt.cam_entries;
                    pt.cam_lanes += (uint64_t)__popcll(__ballot(cam_now));
                    pt.cam_live += (uint64_t)__popcll(__ballot(1));
                }
                uint32_t iters = 0, roots = 0;
                if (cam_now) {
                    ++segs;
                    #ifdef VCRT_COST_MAP  // diagnostics: segments per pixel in the sums' unused fourth channel
                    atomicAdd(P.accum + 4u * (q & kQMask) + 3u, 1.0);
                    #endif
                    // A camera ray starts at the camera centre: its spheres' oc and cc come from
                    // camera-relative records (pair_disc_cam: same bits, half the arithmetic of
                    // pair_disc_cc); the roots take candidate_t_fast.
                    cfloat4* crec = (cfloat4*)P.cam_rec;
                    const float ya = recip_a(aa);
                    const v2f dx = {d.x, d.x}, dy = {d.y, d.y}, dz = {d.z, d.z}, a2 = {aa, aa};
                    for (int gb = 0; gb < P.nbig; ++gb)  // the big spheres (scalar loads)
                        exact_group_uniform_cam(crec + 4 * gb, (cfloat4*)P.cgroup + 5 * gb, dx, dy,
                                                dz, a2, aa, ya, mt, bst, rrow, reg::kCamBig);
                    // the quarter's listed spheres, two per record (primary.cpp): the exact
                    // test's may-hit bits are collected first (bit 2k + s)...
                    const uint32_t cnt = inf & 15u;
                    const float4* lr = P.cam_rec + 4u * (uint32_t)P.nbig + 3u * (inf >> 4);
                    uint32_t cbits = 0u;
                    for (uint32_t k = 0; 2u * k < cnt; ++k) {
                        region(rrow, reg::kCamListTrip);
                        ++iters;
                        const float4 q0 = lr[3u * k], q1 = lr[3u * k + 1u];
                        v2f hb, cc, dc;
                        pair_disc_cam(dx, dy, dz, a2, q0, q1, hb, cc, dc);
                        const uint32_t hits = push_sign(push_sign(0u, hit_sign(hb.y, cc.y, dc.y)),
                                                        hit_sign(hb.x, cc.x, dc.x));
                        cbits |= hits << (2u * k);
                    }
                    // ...then the candidates' roots, one per lane and loop trip (the wave runs
                    // as many trips as its busiest lane has candidates, mostly one), with the
                    // sphere's hb and disc recomputed by the same operations (measured: both
                    // members' roots packed in the first loop issue more VALU, +1.8%)
                    while (cbits) {
                        region(rrow, reg::kCamRootTrip);
                        const uint32_t b = (uint32_t)__builtin_ctz(cbits);
                        cbits &= cbits - 1u;
                        const float4* c = lr + 3u * (b >> 1);
                        const float4 xy = c[0], zc = c[1], id = c[2];
                        const bool hi = (b & 1u) != 0;
                        const float ocx = hi ? xy.y : xy.x, ocy = hi ? xy.w : xy.z;
                        const float ocz = hi ? zc.y : zc.x, cc = hi ? zc.w : zc.z;
                        const float hb = ocx * d.x + ocy * d.y + ocz * d.z;
                        const float disc = hb * hb - aa * cc;
                        consider(candidate_t_fast(hb, disc, aa, ya, rrow),
                                 __float_as_int(hi ? id.y : id.x), mt, bst);
                        ++roots;
                    }
                }
                if constexpr (kStats) {
                    uint32_t tl = iters, tr = roots, ml = iters, mr = roots;
                    for (int off = 32; off > 0; off >>= 1) {
                        tl += (uint32_t)__shfl_xor((int)tl, off);
                        tr += (uint32_t)__shfl_xor((int)tr, off);
                        mr = max(mr, (uint32_t)__shfl_xor((int)mr, off));
                        ml = max(ml, (uint32_t)__shfl_xor((int)ml, off));
                    }
                    pt.list_sum += tl;
                    pt.root_sum += tr;
                    pt.list_trips += ml;
                    pt.root_trips += mr;
                }
                // issued work: the big list and the loop's passes (a pair test is half a group
                // test), per wave
                tally_lds(&ws->work[0], 2u * (uint32_t)P.nbig + wave_max_small<3>(iters));
            }
            // One shading for the camera rays just traced and the main-scan hits of the last
            // iteration: the hit branches run once per iteration for both (a lane has at most
            // one of them; each lane's own sequence of operations is unchanged).
            const bool pending = pend_best != -1;
            if (pending) {
                mt = pend_t;
                bst = pend_best >= 0 ? pend_best : -1;  // kPendSky: the sky
                pend_best = -1;
            }
            uint64_t t_cs = 0;
            if constexpr (kStats) t_cs = ticks();
            if (cam_now || pending) {
                region(rrow, reg::kShadeCam);
                fresh = shade_and_advance(mt, bst, false, reg::kShadeBase0);
            }
            if constexpr (kStats) {
                const uint64_t t1 = ticks();
                pt.cam += t1 - t_cam;
                st_fetch += t1 - t_cs;  // flat stats: debug[3] = the camera phase's shading
            }
            if (need) continue;  // that segment finished the lane's chunk
        }

        // ---- one segment: scan the whole sphere list (functions.glsl:73-81) ----
        ++segs;
        #ifdef VCRT_COST_MAP  // diagnostics: segments per pixel in the sums' unused fourth channel
        atomicAdd(P.accum + 4u * (q & kQMask) + 3u, 1.0);
        #endif
        float max_t = __uint_as_float(vconst<0x47c35000u>());  // kInfinity
        int best = (int)vconst<0xffffffffu>();                   // -1
        uint32_t hit_groups = 0;
        if constexpr (kCull != 0) {
            // culling needs every ray of the wave in the guarded finite range (see above)
            const float aa = dot(d, d);
            const bool guarded = (P.flags & kFlagSceneBounded) != 0 && aa >= 0x1p-20f &&
                                 aa <= 0x1p60f && fabsf(o.x) <= 0x1p30f &&
                                 fabsf(o.y) <= 0x1p30f && fabsf(o.z) <= 0x1p30f;
            if (__ballot(!guarded) == 0) {
                region(rrow, reg::kScan);
                uint32_t lane_cnt = 0;
                uint64_t t0 = 0;
                if constexpr (kStats) t0 = ticks();
                if constexpr (kCull == 1)
                    scan_culled<kStats>(P, o, d, max_t, best, w_halves, w_bounds, hit_groups,
                                        lane_cnt);
                else if constexpr (kFlat)
                    scan_culled_flat<kStats, kFmt, kGRec, kChunks, kNS>(
                        P, tbound, tnode, tg, ws, o, d, pass == 0, q & kQMask, max_t, best, w_halves,
                        w_bounds, pt, rrow);
                else
                    scan_culled_lane<kStats>(P, tbound, tgroup, o, d, max_t, best, w_halves,
                                             w_bounds, lane_cnt, hit_groups);
                if constexpr (kStats) pt.scan += ticks() - t0;
                if constexpr (kStats) {  // CULL stats: debug[3] = sum of per-wave max lane need
                    for (int off = 32; off > 0; off >>= 1)
                        lane_cnt = max(lane_cnt, (uint32_t)__shfl_xor((int)lane_cnt, off));
                    if constexpr (!kFlat) st_fetch += lane_cnt;
                }
            } else {
                region(rrow, reg::kScanLinear);
                scan_spheres<false>(P, lds_geom, n, o, d, max_t, best, hit_groups);
                if constexpr (kFlat)
                    tally_lds(&ws->work[0], 2u * (uint32_t)((n + 3) >> 2));
                else
                    tally(w_halves, 2u * (uint32_t)((n + 3) >> 2));
            }
        } else {
            scan_spheres<kLds>(P, lds_geom, n, o, d, max_t, best, hit_groups);
            tally(w_halves, 2u * (uint32_t)((n + 3) >> 2));
        }
        if constexpr (kStats) st_hitgroups += hit_groups;

        // ---- shade (textures.glsl) or sky (functions.glsl:85-89) ----
        uint64_t t_shade = 0;
        if constexpr (kStats) {
            t_shade = ticks();
            pt.shade_hits += (uint64_t)__popcll(__ballot(best >= 0));
        }
        if constexpr (kFlat) {
            // a hit is shaded with the next iteration's camera rays; so is the sky of a lane
            // whose quantum ended in this iteration's camera phase (its sum in acc awaits the
            // retire, so no second sample may end before it)
            if (best >= 0 || fin) {
                pend_t = max_t;
                pend_best = best >= 0 ? best : kPendSky;
                fresh = false;  // the ray is traced (it may have been a camera ray)
            } else {
                region(rrow, reg::kShadeSkyMain);
                fresh = shade_and_advance(max_t, best, true, reg::kShadeBase1);  // the sky
            }
        } else {
            fresh = shade_and_advance(max_t, best, false, reg::kShadeBase0);
        }
        if constexpr (kStats) pt.shade += ticks() - t_shade;

    }

#ifdef VCRT_WAVE_END_TIMES  // diagnostics builds (VCRT_DEBUG_STATS=2): when waves start, end,
                            // and see the queue drained (s_memrealtime, 100 MHz)
    if (!kStats && lane == 0 && P.debug) {
        const unsigned long long t = __builtin_amdgcn_s_memrealtime();
        atomicMax(P.debug + 4, t);
        atomicMin(P.debug + 5, t);
        atomicAdd(P.debug + 6, t >> 8);
        atomicAdd(P.debug + 7, 1ull);
        atomicMin(P.debug + 9, t_start_rt);
        atomicMin(P.debug + 10, t_drained_rt);
        atomicAdd(P.debug + 11, t_drained_rt >> 8);
        // wave lifetimes in 0.1 ms buckets (debug 12..27, the last open-ended) and how long
        // the wave ran on after it saw the queue drained (28..31: < 0.1, < 0.3, < 0.6 ms, more)
        const unsigned long long life = (t - t_start_rt) / 10000ull;
        atomicAdd(P.debug + 12 + (life < 15ull ? life : 15ull), 1ull);
        const unsigned long long after = t_drained_rt == ~0ull ? 0ull : (t - t_drained_rt) / 10000ull;
        atomicAdd(P.debug + (after < 1ull ? 28 : after < 3ull ? 29 : after < 6ull ? 30 : 31), 1ull);
    }
#endif
    if (ring) {  // the wave's remaining partial sums (every lane of the wave is here)
        __builtin_amdgcn_wave_barrier();
        for (uint32_t i = lane; i < P.ring_n; i += 64u) ring_flush(ring[i], P.accum);
    }
    // one segment-counter atomic per wave
    unsigned long long total = segs;  // widened before the wave sum
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) total += __shfl_xor(total, off);
    if (lane == 0 && total) atomicAdd(P.segments, total);
    if (P.work_done) {  // the tallies' wave sums (64-bit: a wave's total may pass 2^32)
        unsigned long long wh = w_halves, wb = w_bounds;
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) {
            wh += __shfl_xor(wh, off);
            wb += __shfl_xor(wb, off);
        }
        if constexpr (kFlat) {  // and the flat scan's per-wave LDS tallies
            __builtin_amdgcn_wave_barrier();
            wh += ws->work[0];
            wb += ws->work[1];
        }
        if (lane == 0) {
            atomicAdd(P.work_done + 0, wh / 2u);
            atomicAdd(P.work_done + 1, wb);
        }
    }
    if constexpr (kStats) {
        if (lane == 0 && P.debug) {
            atomicAdd(P.debug + 0, (unsigned long long)st_iters);
            atomicAdd(P.debug + 1, (unsigned long long)st_active);
            atomicAdd(P.debug + 2, (unsigned long long)st_hitgroups);
            atomicAdd(P.debug + 3, (unsigned long long)st_fetch);
            const unsigned long long t = __builtin_amdgcn_s_memrealtime();
            atomicMax(P.debug + 4, t);
            atomicMin(P.debug + 5, t);
            atomicAdd(P.debug + 6, t >> 8);  // mean wave end time (in 256-tick units)
            atomicAdd(P.debug + 7, 1ull);
            atomicAdd(P.debug + 8, (unsigned long long)pt.scan);
            atomicAdd(P.debug + 9, (unsigned long long)pt.levels);
            atomicAdd(P.debug + 10, (unsigned long long)pt.node);
            atomicAdd(P.debug + 11, (unsigned long long)pt.group);
            atomicAdd(P.debug + 12, (unsigned long long)pt.cand);
            atomicAdd(P.debug + 13, (unsigned long long)pt.cand_passes);
            atomicAdd(P.debug + 14, (unsigned long long)(ticks() - t_begin));
            atomicAdd(P.debug + 15, (unsigned long long)pt.big);
            atomicAdd(P.debug + 16, (unsigned long long)pt.push);
            atomicAdd(P.debug + 17, (unsigned long long)pt.shade);
            atomicAdd(P.debug + 18, (unsigned long long)pt.fetch);
            atomicAdd(P.debug + 19, (unsigned long long)pt.pass_entries);
            atomicAdd(P.debug + 20, (unsigned long long)pt.pass_lanes);
            atomicAdd(P.debug + 21, (unsigned long long)pt.partial_passes);
            atomicAdd(P.debug + 22, (unsigned long long)pt.passes);
            atomicAdd(P.debug + 23, (unsigned long long)pt.cam);
            atomicAdd(P.debug + 24, (unsigned long long)pt.cam_entries);
            atomicAdd(P.debug + 25, (unsigned long long)pt.cam_lanes);
            atomicAdd(P.debug + 26, (unsigned long long)pt.cam_live);
            atomicAdd(P.debug + 27, (unsigned long long)pt.list_trips);
            atomicAdd(P.debug + 28, (unsigned long long)pt.list_sum);
            atomicAdd(P.debug + 29, (unsigned long long)pt.root_trips);
            atomicAdd(P.debug + 30, (unsigned long long)pt.root_sum);
            atomicAdd(P.debug + 31, (unsigned long long)pt.shade_hits);
            atomicAdd(P.debug + 32, (unsigned long long)pt.retire);
            atomicAdd(P.debug + 33, (unsigned long long)pt.fetch_iters);
            atomicAdd(P.debug + 34, (unsigned long long)pt.blk_fetches);
            atomicAdd(P.debug + 35, (unsigned long long)pt.items_cur);
            atomicAdd(P.debug + 38, (unsigned long long)pt.retire_iters);
            atomicAdd(P.debug + 39, (unsigned long long)pt.quanta);
        }
    }
}
#undef P

}  // namespace

#ifndef VCRT_FLAT_BLOCK
#define VCRT_FLAT_BLOCK 256  // threads per workgroup the LDS flat scan is compiled for
#endif
#ifndef VCRT_FLAT_WAVES
#define VCRT_FLAT_WAVES 5  // waves per SIMD the flat scans are compiled for (LDS allows 5)
#endif

// VCRT_PART selects the kernels of one code-generation unit (Makefile: the global-table flat
// kernels are compiled apart, with the default scheduler settings); unset: every kernel.
#if !defined(VCRT_PART) || VCRT_PART == 1
extern "C" __global__ __launch_bounds__(256) void vcrt_trace_lds(TraceParams p) {
    extern __shared__ __attribute__((aligned(16))) float4 lds_geom[];
    trace_impl<true, false>(p, lds_geom);
}

extern "C" __global__ __launch_bounds__(256) void vcrt_trace_smem(TraceParams p) {
    extern __shared__ __attribute__((aligned(16))) float4 lds_dyn[];
    trace_impl<false, false>(p, lds_dyn);
}

// Culled scan (exact; see scan_culled): spatially grouped sphere table + wave-level group tests.
extern "C" __global__ __launch_bounds__(256) void vcrt_trace_cull(TraceParams p) {
    extern __shared__ __attribute__((aligned(16))) float4 lds_dyn[];
    trace_impl<false, false, 1>(p, lds_dyn);
}

extern "C" __global__ __launch_bounds__(256) void vcrt_trace_cull_stats(TraceParams p) {
    extern __shared__ __attribute__((aligned(16))) float4 lds_dyn[];
    trace_impl<false, true, 1>(p, lds_dyn);
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
extern "C" __global__ __launch_bounds__(VCRT_FLAT_BLOCK)
__attribute__((amdgpu_waves_per_eu(VCRT_FLAT_WAVES))) void vcrt_trace_cull_flat(TraceParams p) {
    extern __shared__ __attribute__((aligned(16))) float4 lds_tab[];
    trace_impl<false, false, 4>(p, lds_tab);
}

// The flat scans' cost-order builds (vcrt_draw_next_frame "cost order"): the product kernel plus
// the per-pixel segment count of the measuring frame and the block order of later frames.
extern "C" __global__ __launch_bounds__(VCRT_FLAT_BLOCK)
__attribute__((amdgpu_waves_per_eu(VCRT_FLAT_WAVES))) void vcrt_trace_cull_flat_cost(TraceParams p) {
    extern __shared__ __attribute__((aligned(16))) float4 lds_tab[];
    trace_impl<false, false, 4, true>(p, lds_tab);
}

extern "C" __global__ __launch_bounds__(256) void vcrt_trace_cull_flat_stats(TraceParams p) {
    extern __shared__ __attribute__((aligned(16))) float4 lds_tab[];
    trace_impl<false, true, 4>(p, lds_tab);
}

#endif

#if !defined(VCRT_PART) || VCRT_PART == 2
// The flat scan for tables too large for LDS beside its stacks (the stress scene): tables in
// global memory (L2-resident), 32-bit stack entries (any group count), stacks alone in LDS.
extern "C" __global__ __launch_bounds__(256)
__attribute__((amdgpu_waves_per_eu(VCRT_FLAT_WAVES))) void vcrt_trace_cull_flat_global(TraceParams p) {
    extern __shared__ __attribute__((aligned(16))) float4 lds_tab[];
    trace_impl<false, false, 5>(p, lds_tab);
}

extern "C" __global__ __launch_bounds__(256)
__attribute__((amdgpu_waves_per_eu(VCRT_FLAT_WAVES))) void vcrt_trace_cull_flat_global_cost(TraceParams p) {
    extern __shared__ __attribute__((aligned(16))) float4 lds_tab[];
    trace_impl<false, false, 5, true>(p, lds_tab);
}

extern "C" __global__ __launch_bounds__(256) void vcrt_trace_cull_flat_global_stats(TraceParams p) {
    extern __shared__ __attribute__((aligned(16))) float4 lds_tab[];
    trace_impl<false, true, 5>(p, lds_tab);
}

// The flat scan for up to 1024 hierarchy groups whose records do not fit in LDS beside the
// stacks (the stress scene): the group and node boxes in LDS, one copy per CU for 16 waves
// (1024-thread workgroups), the group records in global memory, 16-bit stack entries.
extern "C" __global__ __launch_bounds__(1024) void vcrt_trace_cull_flat_boxes(TraceParams p) {
    extern __shared__ __attribute__((aligned(16))) float4 lds_tab[];
    trace_impl<false, false, 6>(p, lds_tab);
}

extern "C" __global__ __launch_bounds__(1024) void vcrt_trace_cull_flat_boxes_cost(TraceParams p) {
    extern __shared__ __attribute__((aligned(16))) float4 lds_tab[];
    trace_impl<false, false, 6, true>(p, lds_tab);
}

extern "C" __global__ __launch_bounds__(1024) void vcrt_trace_cull_flat_boxes_stats(TraceParams p) {
    extern __shared__ __attribute__((aligned(16))) float4 lds_tab[];
    trace_impl<false, true, 6>(p, lds_tab);
}

#endif

#if !defined(VCRT_PART) || VCRT_PART == 1
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
    extern __shared__ __attribute__((aligned(16))) float4 lds_dyn[];
    trace_impl<false, false, 3>(p, lds_dyn);
}

extern "C" __global__ __launch_bounds__(256) void vcrt_trace_cull_lane_stats(TraceParams p) {
    extern __shared__ __attribute__((aligned(16))) float4 lds_dyn[];
    trace_impl<false, true, 3>(p, lds_dyn);
}

// Diagnostics builds (VCRT_DEBUG_STATS=1): same kernels plus lane-occupancy/tail counters.
extern "C" __global__ __launch_bounds__(256) void vcrt_trace_lds_stats(TraceParams p) {
    extern __shared__ __attribute__((aligned(16))) float4 lds_geom[];
    trace_impl<true, true>(p, lds_geom);
}

extern "C" __global__ __launch_bounds__(256) void vcrt_trace_smem_stats(TraceParams p) {
    extern __shared__ __attribute__((aligned(16))) float4 lds_dyn[];
    trace_impl<false, true>(p, lds_dyn);
}

// Exact sample sums -> pixels (vcrt_math.h "Accumulation"; shader.comp:56 divides by SPP).
extern "C" __global__ __launch_bounds__(256) void vcrt_resolve(ResolveParams p) {
    if (p.counters != nullptr && blockIdx.x == 0u) {  // the tracer's counters: read, then zeroed
        unsigned long long v = 0ull;
        if (threadIdx.x < 4u) v = p.counters[threadIdx.x];
        __syncthreads();
        if (threadIdx.x < 4u) p.counters_out[threadIdx.x] = v;
        uint32_t* w = reinterpret_cast<uint32_t*>(p.counters);
        for (uint32_t i = threadIdx.x; i < p.counter_words; i += blockDim.x) w[i] = 0u;
        __threadfence_system();
    }
    const uint32_t elems = p.local_tiles * 64u;
    const double st = (double)p.spp_total, inv_all = p.inv_scale;
    for (uint32_t q = blockIdx.x * blockDim.x + threadIdx.x; q < elems;
         q += gridDim.x * blockDim.x) {
        const Pixel px = pixel_of(q, (uint32_t)p.width, (uint32_t)p.height, p.tiles_x,
                                  (uint32_t)p.world, (uint32_t)p.rank);
        if (!px.valid) continue;
        const double4 s = *reinterpret_cast<const double4*>(p.accum + 4u * q);
        const double inv = p.pixel_emax ? __builtin_ldexp(1.0, -pixel_scale_log2(p.pixel_emax[q]))
                                        : inv_all;
        if (p.zero_accum) *reinterpret_cast<double4*>(p.accum + 4u * q) = double4{0.0, 0.0, 0.0, 0.0};
        p.out[px.out_index] = make_float4(resolve_channel(s.x, inv, st),
                                          resolve_channel(s.y, inv, st),
                                          resolve_channel(s.z, inv, st),
#ifdef VCRT_COST_MAP  // diagnostics: alpha = the pixel's segments (tracer VCRT_COST_MAP)
                                          (float)s.w);
#else
                                          1.0f);
#endif
    }
}

// TraceParams.jitter (SetupJitterParams): the jitter term of every sample index.
extern "C" __global__ __launch_bounds__(256) void vcrt_setup_jitter(SetupJitterParams p) {
    const f3 p00 = mk(p.cam[0], p.cam[1], p.cam[2]);
    const f3 du = mk(p.cam[3], p.cam[4], p.cam[5]);
    const f3 dv = mk(p.cam[6], p.cam[7], p.cam[8]);
    const uint32_t total = p.nsamples + (p.corner ? p.slots : 0u);
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < total;
         i += gridDim.x * blockDim.x) {
        if (i < p.nsamples) {
            const f3 v = viewport_jitter(du, dv, p.jitter_in[i]);
            p.jitter[i] = make_float4(v.x, v.y, v.z, 0.0f);
        } else {  // the pixel corner of local slot q (edge-tile slots outside the frame too)
            const uint32_t q = i - p.nsamples, slot = q & 63u;
            uint32_t tx, ty;
            tile_of(q >> 6, p.rank, p.world, p.tiles_x, &tx, &ty);
            const f3 c = viewport_corner(p00, du, dv, 8u * tx + (slot & 7u), 8u * ty + (slot >> 3));
            p.corner[q] = make_float4(c.x, c.y, c.z, 0.0f);
        }
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

// Self-test of sin_fast (vcrt_math.h) against sin_canonical on the fp32 inputs with bit
// patterns first .. first + count - 1 (wrapping): counts the inputs where they differ and where
// the fast value was not accepted (the fallback ran), and keeps the smallest differing pattern.
extern "C" __global__ __launch_bounds__(256) void vcrt_check_sin(SinCheckParams p) {
    uint64_t bad = 0, fallback = 0;
    uint32_t first_bad = 0xFFFFFFFFu;
    const uint32_t stride = gridDim.x * blockDim.x;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < p.count; i += stride) {
        const uint32_t bits = p.first + i;
        const float x = __uint_as_float(bits);
        float f;
        const bool ok = sin_fast_try(x, f);
        if (!ok) f = sin_canonical(x);
        fallback += ok ? 0u : 1u;
        const float want = sin_canonical(x);
        // and the two-argument form the scatter uses (sin3: sin_fast_try_n<2>), on the input and
        // its negation: every accepted value must be the canonical one
        const float xs[2] = {x, -x};
        float fs[2], ft[2], fu[1];
        const bool ok2 = sin_fast_try_n<2>(xs, fs);
        // and the table form (constants from the kernel arguments, as the tracer reads them)
        const bool okt = sin_fast_try_n<2, true>(xs, ft, (cdouble*)&p.sin_c[0]);
        const bool oku = sin_fast_try_n<1, true>(xs, fu, (cdouble*)&p.sin_c[0]);
        const float wneg = sin_canonical(-x);
        const bool bad2 = (ok2 && (__float_as_uint(fs[0]) != __float_as_uint(want) ||
                                   __float_as_uint(fs[1]) != __float_as_uint(wneg))) ||
                          (okt && (__float_as_uint(ft[0]) != __float_as_uint(want) ||
                                   __float_as_uint(ft[1]) != __float_as_uint(wneg))) ||
                          (oku && __float_as_uint(fu[0]) != __float_as_uint(want));
        if (__float_as_uint(f) != __float_as_uint(want) || bad2) {
            ++bad;
            first_bad = min(first_bad, bits);
        }
    }
    for (int off = 32; off > 0; off >>= 1) {
        bad += __shfl_xor(bad, off);
        fallback += __shfl_xor(fallback, off);
        first_bad = min(first_bad, (uint32_t)__shfl_xor((int)first_bad, off));
    }
    if ((threadIdx.x & 63u) == 0) {
        if (bad) atomicAdd(p.result + 0, (unsigned long long)bad);
        if (fallback) atomicAdd(p.result + 1, (unsigned long long)fallback);
        if (first_bad != 0xFFFFFFFFu) atomicMin(p.first_bad, first_bad);
    }
}

extern "C" __global__ __launch_bounds__(256) void vcrt_fill(FillParams p) {
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < p.count;
         i += gridDim.x * blockDim.x)
        p.out[i] = p.value;
}
#endif
