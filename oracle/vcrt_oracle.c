/* vcrt_oracle.c -- CPU restatement of the reference path tracer.
 *
 * TEST INFRASTRUCTURE ONLY: the parity checker and the cpu_baseline leg of bench.py.
 * Never linked into, or called by, the product library.
 *
 * Parity status (see DESIGN.md section "Oracle"):
 *   - SceneGenerator restatement: PINNED, byte-identical to the reference's own
 *     SceneGenerator.cpp compiled here (oracle/Makefile -> oracle/_ref/SceneGenerator).
 *   - Renderer restatement: the reference's Vulkan render cannot be run here (no Vulkan,
 *     no glslc, no GPU) and its GLSL built-ins are driver-defined, so image parity with the
 *     reference's Vulkan output is UNPINNED. The restatement follows the GLSL line by line
 *     under one canonical fp32 definition of every built-in (below); its math KATs are
 *     checked in tests/test_oracle.py.
 *
 * Canonical math (must match vulkancomputeraytracing_amd/csrc/vcrt_math.h bit for bit):
 *   - IEEE fp32, round to nearest, no FMA contraction (-ffp-contract=off), no FTZ.
 *   - dot(a,b) = (a.x*b.x + a.y*b.y) + a.z*b.z ; length = sqrt(dot) ; normalize = v / length.
 *   - sin(x): x widened to double, reduced (Cody-Waite below 2^20, exact integer
 *     Payne-Hanek above), fdlibm kernel polynomials, rounded once to fp32.
 *   - fract(x) = x - floor(x) (GLSL spec form).
 *   - pow(x, 5) = ((x*x)*(x*x))*x for x >= 0, NaN for x < 0 (GLSL: undefined for x < 0;
 *     Vulkan drivers lower pow to exp2(y*log2 x), which yields NaN there).
 *   - mix(x,y,a) = x*(1-a) + y*a (GLSL spec form).
 *   - undefined return of ray_color after MAX_RECURSION_LEVEL hits -> vec3(0).
 *   - refracted left unset by modified_refract -> vec3(0).
 */
#include "vcrt_oracle.h"

#include <math.h>
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------------------------ */
/* vec3 helpers: every op is one rounded fp32 operation, evaluated left to right.         */

typedef struct { float x, y, z; } v3;

static inline v3 V(float x, float y, float z) { v3 r = {x, y, z}; return r; }
static inline v3 vadd(v3 a, v3 b) { return V(a.x + b.x, a.y + b.y, a.z + b.z); }
static inline v3 vsub(v3 a, v3 b) { return V(a.x - b.x, a.y - b.y, a.z - b.z); }
static inline v3 vmul(v3 a, v3 b) { return V(a.x * b.x, a.y * b.y, a.z * b.z); }
static inline v3 vscale(float s, v3 a) { return V(s * a.x, s * a.y, s * a.z); }
static inline v3 vdivs(v3 a, float s) { return V(a.x / s, a.y / s, a.z / s); }
static inline v3 vneg(v3 a) { return V(-a.x, -a.y, -a.z); }
static inline float vdot(v3 a, v3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
static inline float vlength(v3 a) { return sqrtf(vdot(a, a)); }
static inline v3 vnormalize(v3 a) { float l = vlength(a); return vdivs(a, l); }
/* GLSL cross(x,y) = (x1*y2 - y1*x2, x2*y0 - y2*x0, x0*y1 - y0*x1) */
static inline v3 vcross(v3 a, v3 b) {
    return V(a.y * b.z - b.y * a.z, a.z * b.x - b.z * a.x, a.x * b.y - b.x * a.y);
}
/* GLSL reflect(I,N) = I - 2.0*dot(N,I)*N */
static inline v3 vreflect(v3 i, v3 n) {
    float k = 2.0f * vdot(n, i);
    return vsub(i, vscale(k, n));
}
static inline v3 vload(const float* p) { return V(p[0], p[1], p[2]); }

/* ------------------------------------------------------------------------------------ */
/* canonical sin                                                                          */

static const uint32_t k_two_over_pi_padded[9] = {
    0x00000000u, /* bits of 2/pi above the binary point (none) */
    0xA2F9836Eu, 0x4E441529u, 0xFC2757D1u, 0xF534DDC0u,
    0xDB629599u, 0x3C439041u, 0xFE5163ABu, 0xDEBBC561u};

static const double k_pio2_1 = 1.57079632673412561417e+00;  /* first 33 bits of pi/2 */
static const double k_pio2_1t = 6.07710050650619224932e-11; /* pi/2 - k_pio2_1 */
static const double k_invpio2 = 6.36619772367581382433e-01; /* 2/pi */
static const double k_pio2 = 1.57079632679489661923e+00;

static double ksin(double x) {
    const double S1 = -1.66666666666666324348e-01, S2 = 8.33333333332248946124e-03,
                 S3 = -1.98412698298579493134e-04, S4 = 2.75573137070700676789e-06,
                 S5 = -2.50507602534068634195e-08, S6 = 1.58969099521155010221e-10;
    double z = x * x;
    double v = z * x;
    double r = S2 + z * (S3 + z * (S4 + z * (S5 + z * S6)));
    return x + v * (S1 + z * r);
}

static double kcos(double x) {
    const double C1 = 4.16666666666666019037e-02, C2 = -1.38888888888741095749e-03,
                 C3 = 2.48015872894767294178e-05, C4 = -2.75573143513906633035e-07,
                 C5 = 2.08757232129817482790e-09, C6 = -1.13596475577881948265e-11;
    double z = x * x;
    double r = z * (C1 + z * (C2 + z * (C3 + z * (C4 + z * (C5 + z * C6)))));
    double hz = 0.5 * z;
    double w = 1.0 - hz;
    return w + (((1.0 - w) - hz) + z * r);
}

static uint32_t window32(int bitpos) {
    /* 32 bits of the padded table starting at bit index bitpos (MSB first). */
    int wi = bitpos >> 5, sh = bitpos & 31;
    uint32_t hi = k_two_over_pi_padded[wi];
    if (sh == 0) return hi;
    return (hi << sh) | (k_two_over_pi_padded[wi + 1] >> (32 - sh));
}

float oracle_sin(float xf) {
    uint32_t bits;
    memcpy(&bits, &xf, 4);
    uint32_t e = (bits >> 23) & 0xFFu;
    if (e == 0xFFu) return xf - xf; /* inf, NaN -> NaN */
    double r;
    int q;
    if (e < 147u) { /* |x| < 2^20: Cody-Waite, k*pio2_1 exact (k < 2^20, 33-bit constant) */
        double x = (double)xf;
        double k = rint(x * k_invpio2);
        r = (x - k * k_pio2_1) - k * k_pio2_1t;
        q = (int)((int64_t)k & 3);
    } else { /* exact integer reduction: x = m * 2^s, s >= -3 */
        uint32_t m = (bits & 0x7FFFFFu) | 0x800000u;
        int s = (int)e - 150;
        int b = s + 30; /* bit index of 2/pi bit j = s-1 in the padded table */
        uint64_t w0 = window32(b), w1 = window32(b + 32), w2 = window32(b + 64);
        uint64_t p2 = (uint64_t)m * w2, p1 = (uint64_t)m * w1, p0 = (uint64_t)m * w0;
        uint64_t t = (p2 >> 32) + (p1 & 0xFFFFFFFFu);
        uint32_t mid = (uint32_t)t;
        t = (t >> 32) + (p1 >> 32) + (p0 & 0xFFFFFFFFu);
        uint32_t hi = (uint32_t)t;
        uint64_t frac = ((uint64_t)(hi & 0x3FFFFFFFu) << 34) | ((uint64_t)mid << 2) |
                        ((uint64_t)(uint32_t)p2 >> 30);
        q = (int)(hi >> 30);
        int64_t sf = (int64_t)frac; /* [-0.5,0.5) quadrant fraction, rounds q to nearest */
        if (sf < 0) q += 1;
        r = ((double)sf * 0x1p-64) * k_pio2;
        if (bits >> 31) { r = -r; q = -q; }
        q &= 3;
    }
    double s;
    switch (q & 3) {
        case 0: s = ksin(r); break;
        case 1: s = kcos(r); break;
        case 2: s = -ksin(r); break;
        default: s = -kcos(r); break;
    }
    return (float)s;
}

/* ------------------------------------------------------------------------------------ */
/* The reference's literals, named once (pinned against the reference files by            */
/* tests/golden/reference_constants.json; oracle_reference_constants exports them).        */
#define ORACLE_RAND_DOT_X 12.9898f     /* functions.glsl:11 */
#define ORACLE_RAND_DOT_Y 78.233f      /* functions.glsl:11 */
#define ORACLE_RAND_SCALE 43758.5453f  /* functions.glsl:11 */
#define ORACLE_MIN_T 0.001f            /* functions.glsl:76 */
#define ORACLE_INFINITY 1e5f           /* globals.glsl:26, functions.glsl:75 */
#define ORACLE_SKY_HALF 0.5f           /* functions.glsl:87 */
#define ORACLE_SKY_ONE 1.0f            /* functions.glsl:87 */
#define ORACLE_SKY_BOTTOM 1.0f         /* functions.glsl:88 vec3(1) */
#define ORACLE_SKY_TOP_R 0.5f          /* functions.glsl:88 vec3(.5,.7,1) */
#define ORACLE_SKY_TOP_G 0.7f
#define ORACLE_SKY_TOP_B 1.0f
#define ORACLE_JITTER_OFFSET (-0.5f)   /* shader.comp:48 */

void oracle_reference_constants(float out[ORACLE_NCONSTANTS]) {
    const float c[ORACLE_NCONSTANTS] = {ORACLE_RAND_DOT_X, ORACLE_RAND_DOT_Y, ORACLE_RAND_SCALE,
                                        ORACLE_MIN_T,      ORACLE_INFINITY,   ORACLE_SKY_HALF,
                                        ORACLE_SKY_ONE,    ORACLE_SKY_BOTTOM, ORACLE_SKY_TOP_R,
                                        ORACLE_SKY_TOP_G,  ORACLE_SKY_TOP_B,  ORACLE_JITTER_OFFSET};
    memcpy(out, c, sizeof(c));
}

/* functions.glsl:10-12  rand(co) = fract(sin(dot(co, vec2(12.9898,78.233))) * 43758.5453) */
float oracle_rand(float x, float y) {
    float arg = x * ORACLE_RAND_DOT_X + y * ORACLE_RAND_DOT_Y;
    float p = oracle_sin(arg) * ORACLE_RAND_SCALE;
    return p - floorf(p);
}

/* functions.glsl:42-44: positive-octant "unit sphere" vector seeded by a direction */
static v3 random_in_unit_sphere(v3 seed) {
    return vnormalize(V(oracle_rand(seed.x, seed.y), oracle_rand(seed.x, seed.z),
                        oracle_rand(seed.y, seed.z)));
}

/* functions.glsl:58-62 with canonical pow(x,5) */
static float schlick(float cosine, float ior) {
    float r0 = (1.0f - ior) / (1.0f + ior);
    r0 = r0 * r0;
    float x = 1.0f - cosine;
    float p5 = (x < 0.0f) ? NAN : ((x * x) * (x * x)) * x;
    return r0 + (1.0f - r0) * p5;
}

/* ------------------------------------------------------------------------------------ */
/* camera: shader.comp:18-39                                                              */

static float radians_f(float deg) { return deg * 0.017453292519943295f; }

void oracle_camera(const oracle_config* cfg, float out[15]) {
    v3 lookfrom = vload(cfg->lookfrom), lookat = vload(cfg->lookat), vup = vload(cfg->vup);
    v3 center = lookfrom;
    float focal = vlength(vsub(lookfrom, lookat));
    float theta = radians_f(cfg->vfov);
    float h = (float)tan((double)(theta / 2.0f));
    float vh = 2.0f * h * focal;
    float vw = vh * (float)(cfg->width / cfg->height); /* integer division (shader.comp:25) */
    v3 w = vnormalize(vsub(lookfrom, lookat));
    v3 u = vnormalize(vcross(vup, w));
    v3 v = vcross(w, u);
    v3 viewport_u = vscale(vw, u);
    v3 viewport_v = vscale(vh, vneg(v));
    v3 du = vdivs(viewport_u, (float)cfg->height); /* divided by H (shader.comp:35) */
    v3 dv = vdivs(viewport_v, (float)cfg->height);
    v3 ul = vsub(vsub(vsub(center, vscale(focal, w)), vdivs(viewport_u, 2.0f)),
                 vdivs(viewport_v, 2.0f));
    v3 p00 = vadd(ul, vscale(0.5f, vadd(du, dv)));
    out[0] = p00.x; out[1] = p00.y; out[2] = p00.z;
    out[3] = du.x; out[4] = du.y; out[5] = du.z;
    out[6] = dv.x; out[7] = dv.y; out[8] = dv.z;
    out[9] = center.x; out[10] = center.y; out[11] = center.z;
    out[12] = focal; out[13] = vh; out[14] = vw;
}

/* ------------------------------------------------------------------------------------ */
/* ray_color: functions.glsl:65-92, textures.glsl:19-71                                    */

static v3 ray_color(const oracle_sphere* world, int n, v3 ro, v3 rd, int max_depth,
                    uint64_t* segs) {
    v3 color = V(1.0f, 1.0f, 1.0f);
    for (int pass = 0; pass < max_depth; pass++) {
        (*segs)++;
        float max_t = ORACLE_INFINITY, min_t = ORACLE_MIN_T;
        int hit = 0;
        v3 point = V(0, 0, 0), normal = V(0, 0, 0);
        const oracle_sphere* rec = NULL;
        for (int i = 0; i < n; i++) { /* hit_sphere, functions.glsl:14-40 */
            const oracle_sphere* s = &world[i];
            v3 c = vload(s->center);
            v3 oc = vsub(ro, c);
            float a = vdot(rd, rd);
            float half_b = vdot(oc, rd);
            float cc = vdot(oc, oc) - s->radius * s->radius;
            float disc = half_b * half_b - a * cc;
            if (disc < 0.0f) continue;
            float sq = sqrtf(disc);
            float root = (-half_b - sq) / a;
            if (root <= min_t || max_t <= root) {
                root = (-half_b + sq) / a;
                if (root <= min_t || max_t <= root) continue;
            }
            max_t = root;
            point = vadd(vscale(root, rd), ro);
            normal = vdivs(vsub(point, c), s->radius);
            rec = s;
            hit = 1;
        }
        if (!hit) { /* sky, functions.glsl:85-89 */
            v3 unit = vnormalize(rd);
            float a = ORACLE_SKY_HALF * (unit.y + ORACLE_SKY_ONE);
            float om = 1.0f - a; /* mix(x, y, a) = x * (1 - a) + y * a */
            v3 m = V(ORACLE_SKY_BOTTOM * om + ORACLE_SKY_TOP_R * a,
                     ORACLE_SKY_BOTTOM * om + ORACLE_SKY_TOP_G * a,
                     ORACLE_SKY_BOTTOM * om + ORACLE_SKY_TOP_B * a);
            return vmul(color, m);
        }
        v3 albedo = vload(rec->colour);
        float param = rec->texture[1];
        switch ((int)rec->texture[0]) { /* texture_dispatcher, textures.glsl:65-71 */
            case 1: { /* lambertian, textures.glsl:19-25 */
                v3 dir = vadd(normal, random_in_unit_sphere(rd));
                color = vscale(param, vmul(color, albedo)); /* (colour*albedo)*param */
                ro = point;
                rd = dir;
                break;
            }
            case 2: { /* metal, textures.glsl:58-63 */
                v3 dir = vadd(vreflect(rd, normal), vscale(param, random_in_unit_sphere(rd)));
                color = vmul(color, albedo);
                ro = point;
                rd = dir;
                break;
            }
            case 3: { /* glass, textures.glsl:27-56 */
                v3 reflected = vreflect(rd, normal);
                v3 outward;
                float ni, cosine;
                float dn = vdot(rd, normal);
                if (dn > 0.0f) {
                    outward = vneg(normal);
                    ni = param;
                    cosine = dn;
                    cosine = sqrtf(1.0f - param * param * (1.0f - cosine * cosine));
                } else {
                    outward = normal;
                    ni = 1.0f / param;
                    cosine = -dn;
                }
                v3 refracted = V(0, 0, 0);
                float reflect_prob;
                { /* modified_refract, functions.glsl:46-56 */
                    float dt = vdot(rd, outward);
                    float d = 1.0f - ni * ni * (1.0f - dt * dt);
                    if (d > 0.0f) {
                        float sd = sqrtf(d);
                        refracted = vsub(vscale(ni, vsub(rd, vscale(dt, outward))),
                                         vscale(sd, outward));
                        reflect_prob = schlick(cosine, param);
                    } else {
                        reflect_prob = 1.0f;
                    }
                }
                ro = point;
                rd = (oracle_rand(point.x, point.y) < reflect_prob) ? reflected : refracted;
                break;
            }
            default: /* unknown material: record ignored, ray unchanged */
                break;
        }
    }
    return V(0.0f, 0.0f, 0.0f); /* undefined in GLSL (functions.glsl:92) -> canonical 0 */
}

/* vscale(param, vmul(color, albedo)) computes param*(c*a); GLSL computes (c*a)*param --
 * identical bits since fp32 multiplication is commutative. */

void oracle_ray_color(const oracle_sphere* world, int32_t n, const float origin[3],
                      const float dir[3], int32_t max_depth, float out[3], uint64_t* segments) {
    uint64_t segs = 0;
    v3 c = ray_color(world, n, vload(origin), vload(dir), max_depth, &segs);
    out[0] = c.x; out[1] = c.y; out[2] = c.z;
    if (segments) *segments = segs;
}

/* ------------------------------------------------------------------------------------ */
/* per-pixel driver: shader.comp:42-57, multithreaded over rows or pixels                  */

typedef struct {
    const oracle_config* cfg;
    const oracle_sphere* world;
    int n;
    float* rgba;
    float* seq_rgba; /* optional: the reference's sequential fp32 sum / spp per pixel */
    const float* jitter; /* 2*spp: (-0.5+rand(i,i), -0.5+rand(i+1,i+1)) */
    float cam[15];
    int32_t row_begin, row_end, row_step, nrows;
    const int32_t* pixels; /* pixel-list mode: (x, y) pairs, one output rgba per pair */
    int32_t npixels;
    volatile int next; /* row (or pixel-batch) counter */
    pthread_mutex_t lock;
    uint64_t segments;
    int failed;
} render_job;

/* The quantization scale 2^s of one pixel's run sums (vulkancomputeraytracing_amd/csrc/
 * vcrt_math.h "Accumulation", restated from the rule, not shared code): E = the largest |S| over
 * the channels of the pixel's finite run sums (all progressive frames so far); s = 32 while
 * E < 2^12, else s = 43 - floor(log2 E), the largest s with E * 2^s < 2^44. Every quantized run
 * sum is then an integer below 2^44 and the pixel's at most 512 of them add exactly in double. */
int32_t oracle_pixel_scale_log2(float max_abs) {
    max_abs = fabsf(max_abs);
    if (!(max_abs >= 0x1p12f) || isinf(max_abs)) return 32; /* (only finite sums count) */
    int e;
    (void)frexpf(max_abs, &e); /* max_abs = m * 2^e, m in [0.5, 1): floor(log2) = e - 1 */
    return 43 - (e - 1);
}

/* One pixel (shader.comp:43-57) into px[4] (and the sequential sum into seq[4] if given).
 * Accumulation (vulkancomputeraytracing_amd/csrc/vcrt_math.h "Accumulation"): the samples are
 * cut into quanta of G (accumulate_quantum; before round 4, and still when it is 0, chunks of K
 * plus the tail's chunks), restarting at every progressive frame of frame_spp samples; a quantum
 * is summed in fp32 in sample order, as the reference sums (shader.comp:46-54). A single chunk
 * (K >= spp, no progressive frames) is then divided by SAMPLES_PER_PIXEL in fp32: the
 * reference's own arithmetic (shader.comp:56). Otherwise every quantum sum S is quantized to
 * q = RN_even(S * 2^s) with the pixel's scale (oracle_pixel_scale_log2; a NaN or infinite sum
 * makes the pixel NaN), the q are added exactly (integers below 2^53 in double), and the pixel
 * is (float)((sum * 2^-s) / spp). runs: scratch for 3 floats per run (at most spp runs). */
static void render_pixel(render_job* job, int x, int y, float* px, float* seq, float* runs,
                         uint64_t* segs) {
    const oracle_config* cfg = job->cfg;
    v3 p00 = V(job->cam[0], job->cam[1], job->cam[2]);
    v3 du = V(job->cam[3], job->cam[4], job->cam[5]);
    v3 dv = V(job->cam[6], job->cam[7], job->cam[8]);
    v3 center = V(job->cam[9], job->cam[10], job->cam[11]);
    v3 pc = vadd(vadd(p00, vscale((float)x, du)), vscale((float)y, dv));
    const int block = (cfg->frame_spp <= 0 || cfg->frame_spp > cfg->spp) ? cfg->spp
                                                                        : cfg->frame_spp;
    const int chunk =
        (cfg->accumulate_chunk <= 0 || cfg->accumulate_chunk >= block) ? block
                                                                        : cfg->accumulate_chunk;
    /* the tail: the last `tail` samples of each frame in chunks of tail_chunk, clamped as the
     * product's work_tail clamps explicit values (capi.cpp): at most block - 1 samples, items of
     * at most `tail` samples, none when one chunk covers the frame (no rule here: a tail chunk
     * <= 0 means no tail) */
    const int tail = (cfg->accumulate_tail > 0 && chunk < block && cfg->accumulate_tail_chunk > 0)
                         ? (cfg->accumulate_tail < block ? cfg->accumulate_tail : block - 1)
                         : 0;
    const int tail_chunk =
        cfg->accumulate_tail_chunk < tail ? cfg->accumulate_tail_chunk : tail;
    /* round 4: the accumulation quantum G (> 0) replaces the chunk partition: runs of G samples
     * from each frame's start, whatever the work items (vcrt.h accumulate_quantum) */
    const int quantum = cfg->accumulate_quantum;
    const int single = quantum > 0 ? (cfg->frame_spp <= 0 && quantum >= cfg->spp)
                                   : (cfg->frame_spp <= 0 && chunk >= cfg->spp && tail == 0);
    v3 part = V(0.0f, 0.0f, 0.0f);
    v3 all = V(0.0f, 0.0f, 0.0f); /* the sequential sum (shader.comp:53) */
    int nruns = 0, nan = 0;
    float emax = 0.0f;
    for (int c0 = 0; c0 < cfg->spp;) {
        part = V(0.0f, 0.0f, 0.0f);
        int block_end = (c0 / block + 1) * block;
        if (block_end > cfg->spp) block_end = cfg->spp;
        const int tail_start = block_end - tail;
        int c1;
        if (quantum > 0)
            c1 = c0 + quantum < block_end ? c0 + quantum : block_end;
        else if (c0 < tail_start)
            c1 = c0 + chunk < tail_start ? c0 + chunk : tail_start;
        else
            c1 = c0 + tail_chunk < block_end ? c0 + tail_chunk : block_end;
        for (int i = c0; i < c1; i++) {
            float jx = job->jitter[2 * i], jy = job->jitter[2 * i + 1];
            v3 rs = vadd(vscale(jx, du), vscale(jy, dv));
            v3 ps = vadd(pc, rs);
            v3 dir = vsub(ps, center);
            const v3 rc = ray_color(job->world, job->n, center, dir, cfg->max_depth, segs);
            part = vadd(part, rc);
            all = vadd(all, rc);
        }
        if (!(isfinite(part.x) && isfinite(part.y) && isfinite(part.z))) {
            nan = 1; /* NaN stays NaN through later additions */
        } else {
            const float m = fmaxf(fabsf(part.x), fmaxf(fabsf(part.y), fabsf(part.z)));
            if (m > emax) emax = m;
        }
        runs[3 * nruns + 0] = part.x;
        runs[3 * nruns + 1] = part.y;
        runs[3 * nruns + 2] = part.z;
        nruns++;
        c0 = c1;
    }
    if (single) { /* color /= SAMPLES_PER_PIXEL in fp32 (shader.comp:56) */
        px[0] = part.x / (float)cfg->spp;
        px[1] = part.y / (float)cfg->spp;
        px[2] = part.z / (float)cfg->spp;
    } else if (nan) {
        px[0] = px[1] = px[2] = NAN;
    } else {
        const int32_t s = oracle_pixel_scale_log2(emax);
        const float sc = ldexpf(1.0f, s);
        double sum[3] = {0.0, 0.0, 0.0};
        for (int r = 0; r < nruns; r++)
            for (int k = 0; k < 3; k++) sum[k] += (double)rintf(runs[3 * r + k] * sc);
        for (int k = 0; k < 3; k++)
            px[k] = (float)((sum[k] * ldexp(1.0, -s)) / (double)cfg->spp);
    }
    px[3] = 1.0f;
    if (seq) {
        seq[0] = all.x / (float)cfg->spp;
        seq[1] = all.y / (float)cfg->spp;
        seq[2] = all.z / (float)cfg->spp;
        seq[3] = 1.0f;
    }
}

static void* render_worker(void* arg) {
    render_job* job = (render_job*)arg;
    const oracle_config* cfg = job->cfg;
    uint64_t segs = 0;
    const int batch = 16; /* pixel-list mode hands out pixels 16 at a time */
    const int units = job->pixels ? (job->npixels + batch - 1) / batch : job->nrows;
    float* runs = (float*)malloc(sizeof(float) * 3 * (size_t)cfg->spp);
    if (!runs) {
        pthread_mutex_lock(&job->lock);
        job->failed = 1;
        pthread_mutex_unlock(&job->lock);
        return NULL;
    }
    for (;;) {
        pthread_mutex_lock(&job->lock);
        int k = job->next++;
        pthread_mutex_unlock(&job->lock);
        if (k >= units) break;
        if (job->pixels) {
            for (int p = k * batch; p < job->npixels && p < (k + 1) * batch; p++)
                render_pixel(job, job->pixels[2 * p], job->pixels[2 * p + 1], job->rgba + 4 * p,
                             job->seq_rgba ? job->seq_rgba + 4 * p : NULL, runs, &segs);
        } else {
            int y = job->row_begin + k * job->row_step;
            for (int x = 0; x < cfg->width; x++) {
                const size_t o = ((size_t)y * cfg->width + x) * 4;
                render_pixel(job, x, y, job->rgba + o, job->seq_rgba ? job->seq_rgba + o : NULL,
                             runs, &segs);
            }
        }
    }
    free(runs);
    pthread_mutex_lock(&job->lock);
    job->segments += segs;
    pthread_mutex_unlock(&job->lock);
    return NULL;
}

static int run_job(render_job* job, int32_t threads, uint64_t* segments) {
    const oracle_config* cfg = job->cfg;
    oracle_camera(cfg, job->cam);
    float* jit = (float*)malloc(sizeof(float) * 2 * (size_t)cfg->spp);
    if (!jit) return -1;
    for (int i = 0; i < cfg->spp; i++) {
        jit[2 * i] = ORACLE_JITTER_OFFSET + oracle_rand((float)i, (float)i);
        jit[2 * i + 1] = ORACLE_JITTER_OFFSET + oracle_rand((float)(i + 1), (float)(i + 1));
    }
    job->jitter = jit;
    pthread_mutex_init(&job->lock, NULL);
    if (threads <= 1) {
        render_worker(job);
    } else {
        pthread_t* tids = (pthread_t*)malloc(sizeof(pthread_t) * (size_t)threads);
        int started = 0;
        for (int t = 0; tids && t < threads; t++)
            if (pthread_create(&tids[t], NULL, render_worker, job) == 0) started++;
        if (started == 0) render_worker(job);
        for (int t = 0; t < started; t++) pthread_join(tids[t], NULL);
        free(tids);
    }
    pthread_mutex_destroy(&job->lock);
    free(jit);
    if (job->failed) return -1;
    if (segments) *segments = job->segments;
    return 0;
}

static int config_ok(const oracle_config* cfg) {
    return cfg && cfg->width > 0 && cfg->height > 0 && cfg->spp > 0 && cfg->max_depth >= 0;
}

int oracle_render(const oracle_config* cfg, const oracle_sphere* world, int32_t n, float* rgba,
                  int32_t row_begin, int32_t row_end, int32_t row_step, int32_t threads,
                  uint64_t* segments) {
    return oracle_render_seq(cfg, world, n, rgba, NULL, row_begin, row_end, row_step, threads,
                             segments);
}

int oracle_render_seq(const oracle_config* cfg, const oracle_sphere* world, int32_t n,
                      float* rgba, float* seq_rgba, int32_t row_begin, int32_t row_end,
                      int32_t row_step, int32_t threads, uint64_t* segments) {
    if (!config_ok(cfg) || !rgba || n < 0 || (n > 0 && !world)) return -1;
    if (row_step <= 0) row_step = 1;
    if (row_begin < 0) row_begin = 0;
    if (row_end > cfg->height) row_end = cfg->height;
    render_job job;
    memset(&job, 0, sizeof(job));
    job.cfg = cfg;
    job.world = world;
    job.n = n;
    job.rgba = rgba;
    job.seq_rgba = seq_rgba;
    job.row_begin = row_begin;
    job.row_end = row_end;
    job.row_step = row_step;
    job.nrows = row_end > row_begin ? (row_end - row_begin + row_step - 1) / row_step : 0;
    return run_job(&job, threads, segments);
}

int oracle_render_pixels(const oracle_config* cfg, const oracle_sphere* world, int32_t n,
                         const int32_t* xy, int32_t npixels, float* rgba, int32_t threads,
                         uint64_t* segments) {
    return oracle_render_pixels_seq(cfg, world, n, xy, npixels, rgba, NULL, threads, segments);
}

int oracle_render_pixels_seq(const oracle_config* cfg, const oracle_sphere* world, int32_t n,
                             const int32_t* xy, int32_t npixels, float* rgba, float* seq_rgba,
                             int32_t threads, uint64_t* segments) {
    if (!config_ok(cfg) || npixels < 0 || (npixels > 0 && (!xy || !rgba)) || n < 0 ||
        (n > 0 && !world))
        return -1;
    for (int32_t p = 0; p < npixels; p++)
        if (xy[2 * p] < 0 || xy[2 * p] >= cfg->width || xy[2 * p + 1] < 0 ||
            xy[2 * p + 1] >= cfg->height)
            return -1;
    render_job job;
    memset(&job, 0, sizeof(job));
    job.cfg = cfg;
    job.world = world;
    job.n = n;
    job.rgba = rgba;
    job.seq_rgba = seq_rgba;
    job.pixels = xy;
    job.npixels = npixels;
    return run_job(&job, threads, segments);
}

/* ------------------------------------------------------------------------------------ */
/* presentation encode: linear -> sRGB8 (VK_FORMAT_B8G8R8A8_SRGB store, Frontend.cpp:43)     */

static unsigned char srgb_byte(float c) {
    if (!(c > 0.0f)) return 0; /* negative, zero, NaN */
    if (c >= 1.0f) return 255;
    /* round-to-nearest of 255 * encode(c): the largest k with encode(c) >= (k - 0.5)/255,
     * evaluated as c >= inverse_encode((k - 0.5)/255) in double */
    int lo = 0, hi = 255;
    while (lo < hi) { /* count of thresholds <= c */
        int mid = (lo + hi + 1) / 2;
        double s = (mid - 0.5) / 255.0;
        double lin = s <= 0.04045 ? s / 12.92 : pow((s + 0.055) / 1.055, 2.4);
        if ((double)c >= lin) lo = mid; else hi = mid - 1;
    }
    return (unsigned char)lo;
}

void oracle_encode_srgb8(const float* rgba, size_t pixels, uint8_t* out) {
    for (size_t i = 0; i < pixels; i++) {
        for (int k = 0; k < 3; k++) out[4 * i + k] = srgb_byte(rgba[4 * i + k]);
        float a = rgba[4 * i + 3];
        a = a != a ? 0.0f : (a < 0.0f ? 0.0f : (a > 1.0f ? 1.0f : a));
        out[4 * i + 3] = (uint8_t)(a * 255.0f + 0.5f);
    }
}

/* ------------------------------------------------------------------------------------ */
/* SceneGenerator.cpp restatement: mt19937 (default seed 5489) +                          */
/* libstdc++ generate_canonical<double,53> (two 32-bit draws per double).                 */

typedef struct { uint32_t mt[624]; int idx; } mt19937;

static void mt_seed(mt19937* g, uint32_t s) {
    g->mt[0] = s;
    for (int i = 1; i < 624; i++)
        g->mt[i] = 1812433253u * (g->mt[i - 1] ^ (g->mt[i - 1] >> 30)) + (uint32_t)i;
    g->idx = 624;
}

static uint32_t mt_next(mt19937* g) {
    if (g->idx >= 624) {
        for (int i = 0; i < 624; i++) {
            uint32_t y = (g->mt[i] & 0x80000000u) | (g->mt[(i + 1) % 624] & 0x7FFFFFFFu);
            g->mt[i] = g->mt[(i + 397) % 624] ^ (y >> 1) ^ ((y & 1u) ? 0x9908B0DFu : 0u);
        }
        g->idx = 0;
    }
    uint32_t y = g->mt[g->idx++];
    y ^= y >> 11;
    y ^= (y << 7) & 0x9D2C5680u;
    y ^= (y << 15) & 0xEFC60000u;
    y ^= y >> 18;
    return y;
}

static double random_double(mt19937* g) { /* SceneGenerator.cpp:17-21 */
    double sum = (double)mt_next(g);
    sum += (double)mt_next(g) * 4294967296.0;
    double r = sum / 18446744073709551616.0;
    if (r >= 1.0) r = nextafter(1.0, 0.0);
    return r;
}

typedef struct {
    char* buf;
    size_t cap, len;
} textbuf;

static void tb_printf(textbuf* tb, const char* fmt, ...) __attribute__((format(printf, 2, 3)));
#include <stdarg.h>
static void tb_printf(textbuf* tb, const char* fmt, ...) {
    char tmp[256];
    va_list ap;
    va_start(ap, fmt);
    int k = vsnprintf(tmp, sizeof(tmp), fmt, ap);
    va_end(ap);
    if (k < 0) return;
    if (tb->buf && tb->len + (size_t)k < tb->cap) memcpy(tb->buf + tb->len, tmp, (size_t)k);
    tb->len += (size_t)k;
}

/* One candidate of the generator loop (SceneGenerator.cpp:26-46). GCC evaluates function
 * arguments right to left, so z is drawn before x, and param before b, g, r. Returns 0 if
 * skipped, 1 otherwise; fills the printed text fields. */
typedef struct {
    float cx, cy, cz;
    int kind; /* 1 lambertian, 2 metal, 3 glass */
    double r, g, b, p;
} gen_candidate;

static int gen_one(mt19937* g, int a, int b, gen_candidate* c) {
    double choose = random_double(g);
    double rz = random_double(g);
    double rx = random_double(g);
    c->cx = (float)(a + 0.9 * rx);
    c->cy = (float)0.2;
    c->cz = (float)(b + 0.9 * rz);
    float dx = c->cx - 4.0f, dy = c->cy - (float)0.2, dz = c->cz - 0.0f;
    float len2 = dx * dx + dy * dy + dz * dz; /* vec3::length() is squared (line 14) */
    if ((double)len2 < 0.9) return 0;
    if (choose < 0.8 || choose < 0.95) {
        c->kind = choose < 0.8 ? 1 : 2;
        c->p = random_double(g);
        c->b = random_double(g);
        c->g = random_double(g);
        c->r = random_double(g);
    } else {
        c->kind = 3;
    }
    return 1;
}

size_t oracle_scene_generator_text(char* buf, size_t cap) {
    mt19937 g;
    mt_seed(&g, 5489u);
    textbuf tb = {buf, cap, 0};
    for (int a = -11; a < 11; a++) {
        for (int b = -11; b < 11; b++) {
            gen_candidate c;
            if (!gen_one(&g, a, b, &c)) continue;
            tb_printf(&tb, "sphere(vec3(%.2f,%.2f,%.2f), 0.2, ", (double)c.cx, (double)c.cy,
                      (double)c.cz);
            if (c.kind == 1)
                tb_printf(&tb, "vec3(%.2f,%.2f,%.2f), vec3(TEXTURE_LAMBERTIAN,%.2f,0.0)),\n", c.r,
                          c.g, c.b, c.p);
            else if (c.kind == 2)
                tb_printf(&tb, "vec3(%.2f,%.2f,%.2f), vec3(TEXTURE_METAL,%.2f,0.0)),\n", c.r, c.g,
                          c.b, c.p);
            else
                tb_printf(&tb, "vec3(1.0,1.0,1.0), vec3(TEXTURE_GLASS,1.5,0.0)),\n");
        }
    }
    tb_printf(&tb, "\n");
    tb_printf(&tb, "sphere(vec3(0, 1, 0),1.0, vec3(1.0,1.0,1.0), vec3(TEXTURE_GLASS,1.5,0.0)),\n");
    tb_printf(&tb, "sphere(vec3(-4, 1, 0),1.0, vec3(0.4, 0.2, 0.1), "
                   "vec3(TEXTURE_LAMBERTIAN,1.0,0.0)),\n");
    tb_printf(&tb, "sphere(vec3(4, 1, 0),1.0, vec3(0.7, 0.6, 0.5), "
                   "vec3(TEXTURE_METAL,1.0,0.0)),\n");
    if (buf && cap) buf[tb.len < cap ? tb.len : cap - 1] = '\0';
    return tb.len;
}

static float printed(double v) { /* "%.2f" text parsed back as a GLSL fp32 literal */
    char tmp[64];
    snprintf(tmp, sizeof(tmp), "%.2f", v);
    return strtof(tmp, NULL);
}

int32_t oracle_scene_random_spheres(int32_t lo, int32_t hi, int32_t max_accept,
                                    oracle_sphere* out, int32_t cap) {
    mt19937 g;
    mt_seed(&g, 5489u);
    int32_t count = 0;
    for (int a = lo; a < hi; a++) {
        for (int b = lo; b < hi; b++) {
            if (max_accept > 0 && count >= max_accept) return count;
            gen_candidate c;
            if (!gen_one(&g, a, b, &c)) continue;
            if (count < cap && out) {
                oracle_sphere* s = &out[count];
                s->center[0] = printed((double)c.cx);
                s->center[1] = printed((double)c.cy);
                s->center[2] = printed((double)c.cz);
                s->radius = 0.2f;
                if (c.kind == 3) {
                    s->colour[0] = s->colour[1] = s->colour[2] = 1.0f;
                    s->texture[0] = 3.0f;
                    s->texture[1] = 1.5f;
                } else {
                    s->colour[0] = printed(c.r);
                    s->colour[1] = printed(c.g);
                    s->colour[2] = printed(c.b);
                    s->texture[0] = (float)c.kind;
                    s->texture[1] = printed(c.p);
                }
                s->texture[2] = 0.0f;
            }
            count++;
        }
    }
    return count;
}
