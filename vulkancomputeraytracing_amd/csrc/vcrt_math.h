// vcrt_math.h -- canonical fp32 math shared by the gfx950 tracer kernel and the C++ host
// (camera setup, jitter table). Every function is one fixed sequence of correctly rounded
// IEEE operations, so the device and the host (and the CPU oracle, which restates the same
// definitions independently in oracle/vcrt_oracle.c) agree bit for bit.
//
// The GLSL built-ins these stand for are driver-defined in the reference
// (shaders/include/functions.glsl, textures.glsl); the canonical choices are listed in
// DESIGN.md "Canonical math". Compile with -ffp-contract=off; never with fast-math.
#pragma once

#include <cstdint>

#if defined(__clang__)
#pragma clang fp contract(off)
#endif

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define VCRT_HD __host__ __device__ __forceinline__
#else
#define VCRT_HD inline
#endif

namespace vcrt {

// ---------------------------------------------------------------------------------------
// The reference's literals on the hot path, named once. Pinned against the reference files
// themselves: tests/golden/make_constants_fixture.py parses them into
// tests/golden/reference_constants.json, and tests/test_native_cpu.py checks these definitions,
// the oracle's and vcrt_default_desc against it bit for bit (and that tracer.hip spells none
// of them as a literal).
constexpr float kRandDotX = 12.9898f;      // functions.glsl:11  dot(co, vec2(12.9898, 78.233))
constexpr float kRandDotY = 78.233f;       // functions.glsl:11
constexpr float kRandScale = 43758.5453f;  // functions.glsl:11  sin(...) * 43758.5453
constexpr float kMinT = 0.001f;            // functions.glsl:76  global_hit_record.min_t
constexpr float kInfinity = 1e5f;          // globals.glsl:26, functions.glsl:75: max_t per pass
constexpr float kSkyHalf = 0.5f;           // functions.glsl:87  a = 0.5 * (unit_direction.y + 1.0)
constexpr float kSkyOne = 1.0f;            // functions.glsl:87
constexpr float kSkyBottom = 1.0f;         // functions.glsl:88  mix(vec3(1), vec3(.5,.7,1), a)
constexpr float kSkyTopR = 0.5f, kSkyTopG = 0.7f, kSkyTopB = 1.0f;  // functions.glsl:88
constexpr float kJitterOffset = -0.5f;     // shader.comp:48  (-0.5 + rand(vec2(i,i))) * du + ...
// globals.glsl:9-24 (the `#if 0` resolved: SAMPLES_PER_PIXEL 1), the defaults of vcrt_default_desc
constexpr int32_t kRefSamplesPerPixel = 1, kRefMaxRecursion = 50;
constexpr int32_t kRefImageWidth = 1280, kRefImageHeight = 720;
constexpr float kRefLookfrom[3] = {13.0f, 2.0f, 3.0f}, kRefLookat[3] = {0.0f, 0.0f, 0.0f},
                kRefVup[3] = {0.0f, 1.0f, 0.0f};
constexpr float kRefVfov = 20.0f;

struct f3 {
    float x, y, z;
};

VCRT_HD f3 mk(float x, float y, float z) { return f3{x, y, z}; }
VCRT_HD f3 add(f3 a, f3 b) { return f3{a.x + b.x, a.y + b.y, a.z + b.z}; }
VCRT_HD f3 sub(f3 a, f3 b) { return f3{a.x - b.x, a.y - b.y, a.z - b.z}; }
VCRT_HD f3 mul(f3 a, f3 b) { return f3{a.x * b.x, a.y * b.y, a.z * b.z}; }
VCRT_HD f3 scale(float s, f3 a) { return f3{s * a.x, s * a.y, s * a.z}; }
VCRT_HD f3 divs(f3 a, float s) { return f3{a.x / s, a.y / s, a.z / s}; }
VCRT_HD f3 neg(f3 a) { return f3{-a.x, -a.y, -a.z}; }
// GLSL dot: (x*x' + y*y') + z*z'
VCRT_HD float dot(f3 a, f3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
VCRT_HD float length(f3 a) { return __builtin_sqrtf(dot(a, a)); }
// GLSL normalize(x) = x / length(x)
VCRT_HD f3 normalize(f3 a) { return divs(a, length(a)); }
// GLSL cross(x,y) = (x1*y2 - y1*x2, x2*y0 - y2*x0, x0*y1 - y0*x1)
VCRT_HD f3 cross(f3 a, f3 b) {
    return f3{a.y * b.z - b.y * a.z, a.z * b.x - b.z * a.x, a.x * b.y - b.x * a.y};
}
// GLSL reflect(I,N) = I - 2.0*dot(N,I)*N
VCRT_HD f3 reflect(f3 i, f3 n) { return sub(i, scale(2.0f * dot(n, i), n)); }
VCRT_HD float radians(float deg) { return deg * 0.017453292519943295f; }

// ---------------------------------------------------------------------------------------
// Frame sharding (DESIGN.md "Multi-GPU"): the 8x8 tile (tx, ty) belongs to rank
// (tx + ty) % world, and a rank's tiles are numbered in row-major order (local tile lt).
// Consecutive ranks get consecutive columns of a row, shifted by one per row, so no rank owns a
// whole column of tiles. Every `world` consecutive rows hold exactly tiles_x tiles of each rank.

// Tiles of row ty owned by rank r: the columns tx = s, s + world, ... with s = (r - ty) mod world.
VCRT_HD uint32_t tiles_in_row(uint32_t s, uint32_t tiles_x, uint32_t world) {
    return s < tiles_x ? (tiles_x - 1u - s) / world + 1u : 0u;
}

// Local tile lt of rank r -> (tx, ty).
VCRT_HD void tile_of(uint32_t lt, uint32_t r, uint32_t world, uint32_t tiles_x, uint32_t* tx,
                     uint32_t* ty) {
    const uint32_t period = lt / tiles_x;
    uint32_t rem = lt - period * tiles_x, row = period * world, s = r;  // row % world == 0
    for (;;) {
        const uint32_t c = tiles_in_row(s, tiles_x, world);
        if (rem < c) break;
        rem -= c;
        ++row;
        s = s == 0u ? world - 1u : s - 1u;
    }
    *tx = s + world * rem;
    *ty = row;
}

// Tile (tx, ty) -> its rank and local tile index.
VCRT_HD void owner_of(uint32_t tx, uint32_t ty, uint32_t world, uint32_t tiles_x, uint32_t* r,
                      uint32_t* lt) {
    const uint32_t rank = (tx + ty) % world;
    const uint32_t j = ty % world;
    uint32_t n = (ty / world) * tiles_x, s = rank;
    for (uint32_t k = 0; k < j; ++k) {  // rows ty - j .. ty - 1 of this period
        n += tiles_in_row(s, tiles_x, world);
        s = s == 0u ? world - 1u : s - 1u;
    }
    *r = rank;
    *lt = n + tx / world;
}

// ---------------------------------------------------------------------------------------
// canonical sin: fp32 argument widened to double, reduced to [-pi/4, pi/4] (Cody-Waite for
// |x| < 2^20, exact 96-bit integer reduction by 2/pi above), fdlibm kernels, one rounding.
// Equals the correctly rounded sinf except in astronomically rare double-rounding ties
// (tests/test_oracle.py checks it against float64 sin on 4e5 arguments).

VCRT_HD double ksin(double x) {
    const double S1 = -1.66666666666666324348e-01, S2 = 8.33333333332248946124e-03,
                 S3 = -1.98412698298579493134e-04, S4 = 2.75573137070700676789e-06,
                 S5 = -2.50507602534068634195e-08, S6 = 1.58969099521155010221e-10;
    double z = x * x;
    double v = z * x;
    double r = S2 + z * (S3 + z * (S4 + z * (S5 + z * S6)));
    return x + v * (S1 + z * r);
}

VCRT_HD double kcos(double x) {
    const double C1 = 4.16666666666666019037e-02, C2 = -1.38888888888741095749e-03,
                 C3 = 2.48015872894767294178e-05, C4 = -2.75573143513906633035e-07,
                 C5 = 2.08757232129817482790e-09, C6 = -1.13596475577881948265e-11;
    double z = x * x;
    double r = z * (C1 + z * (C2 + z * (C3 + z * (C4 + z * (C5 + z * C6)))));
    double hz = 0.5 * z;
    double w = 1.0 - hz;
    return w + (((1.0 - w) - hz) + z * r);
}

// 32-bit windows of 2/pi = 0.A2F9836E 4E441529 ..., with one zero word in front.
VCRT_HD uint32_t two_over_pi_word(int i) {
    switch (i) {
        case 0: return 0x00000000u;
        case 1: return 0xA2F9836Eu;
        case 2: return 0x4E441529u;
        case 3: return 0xFC2757D1u;
        case 4: return 0xF534DDC0u;
        case 5: return 0xDB629599u;
        case 6: return 0x3C439041u;
        case 7: return 0xFE5163ABu;
        default: return 0xDEBBC561u;
    }
}

VCRT_HD uint32_t two_over_pi_window(int bitpos) {
    int wi = bitpos >> 5, sh = bitpos & 31;
    uint32_t hi = two_over_pi_word(wi);
    if (sh == 0) return hi;
    return (hi << sh) | (two_over_pi_word(wi + 1) >> (32 - sh));
}

// Large-argument reduction (|x| >= 2^20): r in [-pi/4, pi/4), quadrant q in [0,4).
VCRT_HD double reduce_large(uint32_t bits, int* q_out) {
    uint32_t e = (bits >> 23) & 0xFFu;
    uint32_t m = (bits & 0x7FFFFFu) | 0x800000u;
    int b = (int)e - 150 + 30;
    uint64_t w0 = two_over_pi_window(b), w1 = two_over_pi_window(b + 32),
             w2 = two_over_pi_window(b + 64);
    uint64_t p2 = (uint64_t)m * w2, p1 = (uint64_t)m * w1, p0 = (uint64_t)m * w0;
    uint64_t t = (p2 >> 32) + (p1 & 0xFFFFFFFFu);
    uint32_t mid = (uint32_t)t;
    t = (t >> 32) + (p1 >> 32) + (p0 & 0xFFFFFFFFu);
    uint32_t hi = (uint32_t)t;
    uint64_t frac = ((uint64_t)(hi & 0x3FFFFFFFu) << 34) | ((uint64_t)mid << 2) |
                    ((uint64_t)(uint32_t)p2 >> 30);
    int q = (int)(hi >> 30);
    int64_t sf = (int64_t)frac;
    if (sf < 0) q += 1;
    double r = ((double)sf * 0x1p-64) * 1.57079632679489661923e+00;
    if (bits >> 31) {
        r = -r;
        q = -q;
    }
    *q_out = q & 3;
    return r;
}

VCRT_HD float sin_canonical(float xf) {
    uint32_t bits = __builtin_bit_cast(uint32_t, xf);
    uint32_t e = (bits >> 23) & 0xFFu;
    if (e == 0xFFu) return xf - xf;
    double r;
    int q;
    if (e < 147u) {
        double x = (double)xf;
        double k = __builtin_rint(x * 6.36619772367581382433e-01);
        r = (x - k * 1.57079632673412561417e+00) - k * 6.07710050650619224932e-11;
        q = (int)((int64_t)k & 3);
    } else {
        r = reduce_large(bits, &q);
    }
    double s = (q & 1) ? kcos(r) : ksin(r);
    if (q & 2) s = -s;
    return (float)s;
}

// The fast sine's constants in the order sin_fast_try_n reads them from a table (kTab): 1/pi,
// the 1.5 * 2^52 shifter, pi_hi, pi_mid, then (-1)^j / (2j+1)! for j = 9 .. 1. The host copies
// them into TraceParams.sin_c; the literals in sin_fast_try_n are the same values.
constexpr double kSinC[13] = {0.31830988618379067154, 0x1.8p52, 0x1.921fb544p+1,
                              0x1.0b4611a626331p-33, -0x1.2f49b46814157p-57,
                              0x1.952c77030ad4ap-49, -0x1.ae7f3e733b81fp-41,
                              0x1.6124613a86d09p-33, -0x1.ae64567f544e4p-26,
                              0x1.71de3a556c734p-19, -0x1.a01a01a01a01ap-13,
                              0x1.1111111111111p-7, -0x1.5555555555555p-3};

#if defined(__HIP_DEVICE_COMPILE__)
// The canonical sin on the device, by Ziv's method: one branch-free evaluation for every lane
// (sin_canonical evaluates both fdlibm kernels under divergence, since the quadrant varies per
// lane), accepted when it provably rounds to the same fp32 as sin_canonical, else
// sin_canonical itself. Fast value s: x reduced modulo pi (k = rint(x / pi); r = x - k pi with
// pi split as pi_hi (33 bits: k pi_hi exact for |k| < 2^20) + pi_mid, FMAs), then Taylor to
// r^19 on |r| <= pi/2 (truncation < 2^-51.8 |sin r|), sign (-1)^k. For |x| < 2^19 and
// |r| >= 2^-12 the error of s and that of sin_canonical's double result (2-term Cody-Waite
// reduction, fdlibm kernels)
// are each below 2^-48 |sin x|; if s lies farther than 2^-44 |s| from every fp32 rounding
// boundary, both round to the same float f. Otherwise (|r| < 2^-12, |x| >= 2^19, or s near a
// boundary: ~2e-4 of the calls) the lane takes sin_canonical.
// tests/test_gpu_parity.py::test_sin_fast_exhaustive compares the two on all 2^32 inputs.
// A double constant materialised in an SGPR pair where it is used: plain literals get hoisted
// out of the tracer's loops into VGPR pairs, which then spill (v_fma_f64 takes no 64-bit
// literal on gfx950).
template <uint64_t kBits>
__device__ __forceinline__ double sconst() {
    uint32_t lo, hi;
    asm volatile("s_mov_b32 %0, %1" : "=s"(lo) : "i"((uint32_t)kBits));
    asm volatile("s_mov_b32 %0, %1" : "=s"(hi) : "i"((uint32_t)(kBits >> 32)));
    return __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
}
#define VCRT_DC(x) sconst<__builtin_bit_cast(uint64_t, (double)(x))>()

// fma(a, b, c) with c an SGPR pair, as one VOP3 v_fma_f64. The compiler otherwise picks the
// two-address v_fmac_f64, which needs the addend in the destination: two v_mov_b32 per
// Horner step of sin_fast_try (20 of its ~45 VALU instructions).
__device__ __forceinline__ double fma_vvs(double a, double b, double c) {
    double d;
    asm("v_fma_f64 %0, %1, %2, %3" : "=v"(d) : "v"(a), "v"(b), "s"(c));
    return d;
}

// Round 2: k by the 1.5 * 2^52 shifter (t = x / pi + 1.5 * 2^52 in one FMA: t's last mantissa
// bit is k's parity, which flips the sign), and the boundary test on s's own mantissa: in s's
// binade the fp32 rounding boundaries sit where the 29 bits below fp32 precision equal 2^28, so
// s is accepted when those bits differ from 2^28 by more than 2^9 units of s's last place
// (2^9 ulp_double(s) >= 2^-44 |s|, the margin above; binade ends need no special case).
__device__ __forceinline__ bool sin_fast_try(float xf, float& out) {
    const double x = (double)xf;
    const double t = __builtin_fma(x, VCRT_DC(0.31830988618379067154), VCRT_DC(0x1.8p52));
    const double k = t - VCRT_DC(0x1.8p52);
    double r = __builtin_fma(-k, VCRT_DC(0x1.921fb544p+1), x);
    r = __builtin_fma(-k, VCRT_DC(0x1.0b4611a626331p-33), r);
    const double r2 = r * r;
    double p = VCRT_DC(-0x1.2f49b46814157p-57);  // (-1)^j / (2j+1)!, j = 9 .. 1
    p = fma_vvs(p, r2, VCRT_DC(0x1.952c77030ad4ap-49));
    p = fma_vvs(p, r2, VCRT_DC(-0x1.ae7f3e733b81fp-41));
    p = fma_vvs(p, r2, VCRT_DC(0x1.6124613a86d09p-33));
    p = fma_vvs(p, r2, VCRT_DC(-0x1.ae64567f544e4p-26));
    p = fma_vvs(p, r2, VCRT_DC(0x1.71de3a556c734p-19));
    p = fma_vvs(p, r2, VCRT_DC(-0x1.a01a01a01a01ap-13));
    p = fma_vvs(p, r2, VCRT_DC(0x1.1111111111111p-7));
    p = fma_vvs(p, r2, VCRT_DC(-0x1.5555555555555p-3));
    double s = __builtin_fma(r * r2, p, r);
    const uint64_t tb = __builtin_bit_cast(uint64_t, t);
    const uint64_t sb = __builtin_bit_cast(uint64_t, s) ^ (tb << 63);  // (-1)^k
    out = (float)__builtin_bit_cast(double, sb);
    // bits 28..0 of s's mantissa (|s| >= 2^-13: normal in both formats)
    const uint32_t below = (uint32_t)sb & 0x1FFFFFFFu;
    const bool ok = __builtin_fabsf(xf) < 0x1p19f && __builtin_fabs(r) >= 0x1p-12 &&
                    below - (0x10000000u - 0x200u) > 0x400u;
    return ok;
}

// sin_fast_try of N arguments at once, step by step: each constant is materialized once and
// used by the N evaluations (sconst's two s_mov_b32 per use were ~90 SALU instructions per
// scatter with three separate calls), each argument's operations unchanged.
typedef __attribute__((address_space(4))) const double cdouble;
template <int N, bool kTab = false>
__device__ __forceinline__ bool sin_fast_try_n(const float* xf, float* out,
                                               cdouble* kc = nullptr) {
#define VCRT_SC(j, lit)                                 \
    ([&]() -> double {                                  \
        if constexpr (kTab)                             \
            return kc[j];                               \
        else                                            \
            return VCRT_DC(lit);                        \
    }())
    double x[N], t[N], k[N], r[N], r2[N], p[N];
    for (int i = 0; i < N; ++i) x[i] = (double)xf[i];
    {
        const double c = VCRT_SC(0, 0.31830988618379067154), sh = VCRT_SC(1, 0x1.8p52);
        for (int i = 0; i < N; ++i) t[i] = __builtin_fma(x[i], c, sh);
        for (int i = 0; i < N; ++i) k[i] = t[i] - sh;
    }
    {
        const double c = VCRT_SC(2, 0x1.921fb544p+1);
        for (int i = 0; i < N; ++i) r[i] = __builtin_fma(-k[i], c, x[i]);
    }
    {
        const double c = VCRT_SC(3, 0x1.0b4611a626331p-33);
        for (int i = 0; i < N; ++i) r[i] = __builtin_fma(-k[i], c, r[i]);
    }
    for (int i = 0; i < N; ++i) r2[i] = r[i] * r[i];
    {
        const double c = VCRT_SC(4, -0x1.2f49b46814157p-57);  // (-1)^j / (2j+1)!, j = 9 .. 1
        for (int i = 0; i < N; ++i) p[i] = c;
    }
#define VCRT_SIN3_STEP(J, C)                                               \
    {                                                                      \
        const double c = VCRT_SC(J, C);                                    \
        for (int i = 0; i < N; ++i) p[i] = fma_vvs(p[i], r2[i], c);        \
    }
    VCRT_SIN3_STEP(5, 0x1.952c77030ad4ap-49)
    VCRT_SIN3_STEP(6, -0x1.ae7f3e733b81fp-41)
    VCRT_SIN3_STEP(7, 0x1.6124613a86d09p-33)
    VCRT_SIN3_STEP(8, -0x1.ae64567f544e4p-26)
    VCRT_SIN3_STEP(9, 0x1.71de3a556c734p-19)
    VCRT_SIN3_STEP(10, -0x1.a01a01a01a01ap-13)
    VCRT_SIN3_STEP(11, 0x1.1111111111111p-7)
    VCRT_SIN3_STEP(12, -0x1.5555555555555p-3)
#undef VCRT_SIN3_STEP
#undef VCRT_SC
    bool ok = true;
    for (int i = 0; i < N; ++i) {
        const double s = __builtin_fma(r[i] * r2[i], p[i], r[i]);
        const uint64_t tb = __builtin_bit_cast(uint64_t, t[i]);
        const uint64_t sb = __builtin_bit_cast(uint64_t, s) ^ (tb << 63);  // (-1)^k
        out[i] = (float)__builtin_bit_cast(double, sb);
        const uint32_t below = (uint32_t)sb & 0x1FFFFFFFu;
        ok = ok && __builtin_fabsf(xf[i]) < 0x1p19f && __builtin_fabs(r[i]) >= 0x1p-12 &&
             below - (0x10000000u - 0x200u) > 0x400u;
    }
    return ok;
}

// The three rand() values of a scatter (textures.glsl:21, :51, functions.glsl:43): sines of
// a1, a2 by sin_fast_try_n<2> (shared constants: measured +1.0% at C4, +1.5-3% at C2 against
// three separate calls; all three interleaved spilled a loop counter), a3 by sin_fast_try; a
// lane whose fast values were not all accepted recomputes all three
// canonically in one loop (one inlined copy of the fdlibm path instead of three).
template <bool kTab = false>
__device__ __forceinline__ void sin3(float a1, float a2, float a3, float& s1, float& s2,
                                     float& s3, cdouble* kc = nullptr, bool* fell_back = nullptr) {
    const float a[2] = {a1, a2};
    float sv[2];
    bool ok = sin_fast_try_n<2, kTab>(a, sv, kc);
    if constexpr (kTab) {
        const float a3v[1] = {a3};
        float s3v[1];
        ok = ok & sin_fast_try_n<1, true>(a3v, s3v, kc);
        s3 = s3v[0];
    } else {
        ok = ok & sin_fast_try(a3, s3);
    }
    s1 = sv[0];
    s2 = sv[1];
    if (fell_back) *fell_back = !ok;  // stats builds (tracer.hip region counters)
    if (!ok) {
#pragma nounroll
        for (int j = 0; j < 3; ++j) {
            const float c = sin_canonical(j == 0 ? a1 : j == 1 ? a2 : a3);
            s1 = j == 0 ? c : s1;
            s2 = j == 1 ? c : s2;
            s3 = j == 2 ? c : s3;
        }
    }
}

__device__ __forceinline__ float sin_fast(float xf) {
    float f;
    if (!sin_fast_try(xf, f)) f = sin_canonical(xf);
    return f;
}
#endif

// functions.glsl:10-12  rand(co) = fract(sin(dot(co, vec2(12.9898,78.233))) * 43758.5453),
// split as the sine's argument and the fract of the scaled sine
VCRT_HD float rand_arg(float x, float y) { return x * kRandDotX + y * kRandDotY; }
VCRT_HD float rand_of_sin(float s) {
    const float p = s * kRandScale;
    return p - __builtin_floorf(p);
}

VCRT_HD float rand2(float x, float y) {
    float arg = rand_arg(x, y);
#if defined(__HIP_DEVICE_COMPILE__)
    float p = sin_fast(arg) * kRandScale;
#else
    float p = sin_canonical(arg) * kRandScale;
#endif
    return p - __builtin_floorf(p);
}

// functions.glsl:85-88: the sky's factor mix(vec3(1), vec3(.5,.7,1), 0.5 * (y / |d| + 1)) for
// the segment's direction d (not normalised first: y / length(d) is unit_direction.y)
VCRT_HD f3 sky_factor(float y_over_len) {
    const float t = kSkyHalf * (y_over_len + kSkyOne);
    const float om = 1.0f - t;  // GLSL mix(x, y, a) = x * (1 - a) + y * a
    return f3{kSkyBottom * om + kSkyTopR * t, kSkyBottom * om + kSkyTopG * t,
              kSkyBottom * om + kSkyTopB * t};
}

// functions.glsl:58-62 with canonical pow(x,5): NaN for x < 0 (GLSL leaves it undefined)
VCRT_HD float schlick(float cosine, float ior) {
    float r0 = (1.0f - ior) / (1.0f + ior);
    r0 = r0 * r0;
    float x = 1.0f - cosine;
    float p5 = (x < 0.0f) ? __builtin_nanf("") : ((x * x) * (x * x)) * x;
    return r0 + (1.0f - r0) * p5;
}

// schlick with r0 = ((1 - ior) / (1 + ior))^2 given (the same operations as schlick after it)
VCRT_HD float schlick_r0(float cosine, float r0) {
    float x = 1.0f - cosine;
    float p5 = (x < 0.0f) ? __builtin_nanf("") : ((x * x) * (x * x)) * x;
    return r0 + (1.0f - r0) * p5;
}

// ---------------------------------------------------------------------------------------
// Accumulation (shader.comp:46-56: color.rgb += ray_color(...); color /= SPP). The reference
// sums a pixel's samples in fp32 in sample order. The GPU cuts them into quanta of G
// consecutive samples (the accumulation quantum, restarting at every progressive frame; work
// items hold whole quanta) and sums each quantum the same way. One quantum per pixel (G >= spp,
// not progressive): color / SPP in fp32, the reference's arithmetic exactly. Otherwise each
// quantum sum S is quantized to q = RN_even(S * 2^s) (the scaling is exact), the q are added in
// double -- exact, as |q| < 2^44 and a pixel has at most 512 quanta (< 2^53) -- and
//     out = (float)((sum * 2^-s) / (double)spp_total).
// Exact sums do not depend on the order of the additions, so the image depends on G and s
// alone: not on the work items, the schedule or the number of GPUs (a sharded frame equals the
// one-GPU frame bit for bit). The scale 2^s is per pixel (pixel_scale_log2), from E, the
// largest |S| of the pixel's finite quantum sums (every channel, every progressive frame so
// far): s = 32 while E < 2^12 -- every pixel of the reference scenes, whose radiance is <= 1 per
// sample, which keeps every S >= 2^-9 exactly -- else the largest s with E * 2^s < 2^44. A pixel
// depends on its own samples only, so any rank computes its scale alone. The kernel quantizes at
// the scale it was given (32, or the pixel's from TraceParams.pixel_emax); a quantum with
// |S * 2^s| >= 2^44 records max|S| there (atomicMax on the float bits) and the host renders the
// frame again with every pixel at its own scale (capi.cpp "Outlier quanta"). A NaN or infinite
// quantum sum makes the pixel NaN. The quantized combination differs from the fp32 sequential
// sum by less than that sum's own rounding error.
constexpr int32_t kAccumMaxScaleLog2 = 32;
constexpr float kAccumQLimit = 0x1p44f;   // |q| bound of one quantum sum
constexpr int32_t kAccumMaxChunks = 512;  // quanta per pixel (progressive frames included)

// The scale s of a pixel whose largest finite |quantum sum| has the float bits emax_bits (0: none
// reached 2^12): 32, or 43 - floor(log2 E) = 170 - biased exponent (E >= 2^12 is normal).
VCRT_HD int32_t pixel_scale_log2(uint32_t emax_bits) {
    return emax_bits == 0u ? kAccumMaxScaleLog2 : 170 - static_cast<int32_t>(emax_bits >> 23);
}

// One channel of a pixel from the exact sum of its quantized quantum sums; inv_scale = 2^-s.
VCRT_HD float resolve_channel(double s, double inv_scale, double spp_total) {
    return (float)((s * inv_scale) / spp_total);
}

// ---------------------------------------------------------------------------------------
// Camera: shader.comp:18-39, computed once on the host (it is uniform per dispatch).

struct Camera {
    f3 pixel00, delta_u, delta_v, center;
    float focal_length, viewport_height, viewport_width;
};

inline Camera make_camera(int width, int height, f3 lookfrom, f3 lookat, f3 vup, float vfov,
                          double (*tan_fn)(double)) {
    Camera c;
    c.center = lookfrom;
    c.focal_length = length(sub(lookfrom, lookat));
    float theta = radians(vfov);
    float h = (float)tan_fn((double)(theta / 2.0f));
    c.viewport_height = 2.0f * h * c.focal_length;
    c.viewport_width = c.viewport_height * (float)(width / height);  // integer division
    f3 w = normalize(sub(lookfrom, lookat));
    f3 u = normalize(cross(vup, w));
    f3 v = cross(w, u);
    f3 viewport_u = scale(c.viewport_width, u);
    f3 viewport_v = scale(c.viewport_height, neg(v));
    c.delta_u = divs(viewport_u, (float)height);  // divided by H (shader.comp:35)
    c.delta_v = divs(viewport_v, (float)height);
    f3 ul = sub(sub(sub(c.center, scale(c.focal_length, w)), divs(viewport_u, 2.0f)),
                divs(viewport_v, 2.0f));
    c.pixel00 = add(ul, scale(0.5f, add(c.delta_u, c.delta_v)));
    return c;
}

}  // namespace vcrt
