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
//   * One pixel per lane, all of its samples in sample order (so the fp32 sum is the
//     reference's sequential sum, bit for bit). A lane whose path ends starts its next
//     sample at once (path regeneration) and a lane whose pixel is done takes the next pixel
//     from a wave-aggregated atomic work counter, so lanes stay busy until the queue drains.
//   * Ray state lives in VGPRs. The sphere list (center, r^2) is staged once per workgroup in
//     LDS (kLds) or read through the scalar cache with wave-uniform s_load (!kLds); either way
//     every lane tests sphere j at the same time, so the data is a broadcast.
//   * Only fp32 add/sub/mul plus correctly rounded div/sqrt, no contraction: the results are
//     bit-identical to the CPU oracle. No MFMA (branchy scalar math, not a contraction).
#include <hip/hip_runtime.h>

#include "vcrt_kernel_abi.h"
#include "vcrt_math.h"

#pragma clang fp contract(off)

using namespace vcrt;

namespace {

constexpr int kBand = 8;  // rows per work band (8x8 tiles of 64 consecutive items)

__device__ __forceinline__ uint32_t lanes_below(uint64_t mask) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32),
                                     __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u));
}

typedef __attribute__((address_space(4))) const float4 cfloat4;

template <bool kLds>
__device__ __forceinline__ float4 sphere_geom(const float4* lds, const TraceParams& p, int j) {
    if constexpr (kLds) {
        return lds[j];
    } else {
        return ((cfloat4*)p.geom)[j];  // uniform index -> s_load through the scalar cache
    }
}

template <bool kLds>
__device__ __forceinline__ void trace_impl(const TraceParams& p, float4* lds_geom) {
    const int n = p.nspheres;
    if constexpr (kLds) {
        for (int i = threadIdx.x; i < n; i += blockDim.x) lds_geom[i] = p.geom[i];
        __syncthreads();
    }
    const uint32_t lane = threadIdx.x & 63u;
    const f3 p00 = mk(p.cam[0], p.cam[1], p.cam[2]);
    const f3 du = mk(p.cam[3], p.cam[4], p.cam[5]);
    const f3 dv = mk(p.cam[6], p.cam[7], p.cam[8]);
    const f3 cam = mk(p.cam[9], p.cam[10], p.cam[11]);
    const float spp_f = (float)p.spp;
    const uint32_t W = (uint32_t)p.width;
    const float min_t = 0.001f;

    bool done = false, need = true;
    int sample = 0, pass = 0;
    uint32_t out_index = 0;
    f3 pc = mk(0.f, 0.f, 0.f), o = pc, d = pc, atten = pc, acc = pc;
    unsigned long long segs = 0;

    for (;;) {
        // ---- take new pixels for lanes that finished theirs (one atomic per wave) ----
        const uint64_t need_mask = __ballot(need && !done);
        if (need_mask) {
            const int leader = __ffsll((unsigned long long)need_mask) - 1;
            uint32_t base = 0;
            if ((int)lane == leader) base = atomicAdd(p.work, (uint32_t)__popcll(need_mask));
            base = __shfl(base, leader);
            if (need && !done) {
                const uint32_t item = base + lanes_below(need_mask);
                if (item >= p.total_items) {
                    done = true;
                } else {
                    const uint32_t band = item / (kBand * W);
                    const uint32_t r = item - band * kBand * W;
                    const uint32_t rows_left = (uint32_t)p.local_rows - band * kBand;
                    const uint32_t rows_in_band = rows_left < kBand ? rows_left : kBand;
                    const uint32_t x = r / rows_in_band;
                    const uint32_t lr = band * kBand + (r - x * rows_in_band);
                    const uint32_t ls = lr / (uint32_t)p.stripe_h;
                    const uint32_t within = lr - ls * (uint32_t)p.stripe_h;
                    const uint32_t y =
                        (ls * (uint32_t)p.world + (uint32_t)p.rank) * (uint32_t)p.stripe_h + within;
                    out_index = lr * W + x;
                    // shader.comp:43  pixel00 + x*delta_u + y*delta_v
                    pc = add(add(p00, scale((float)x, du)), scale((float)y, dv));
                    acc = mk(0.f, 0.f, 0.f);
                    sample = 0;
                    // first camera ray, shader.comp:48-52
                    const float2 jt = p.jitter[0];
                    const f3 ps = add(pc, add(scale(jt.x, du), scale(jt.y, dv)));
                    o = cam;
                    d = sub(ps, cam);
                    atten = mk(1.f, 1.f, 1.f);
                    pass = 0;
                }
                need = false;
            }
        }
        if (__ballot(!done) == 0) break;
        if (done) continue;

        // ---- one segment: scan the whole sphere list (functions.glsl:73-81) ----
        ++segs;
        const float a = dot(d, d);  // loop-invariant in hit_sphere: hoisting is exact
        float max_t = 1e5f;
        int best = -1;
        int j = 0;
        const int n4 = n & ~3;
        for (; j < n4; j += 4) {
            float hb[4], disc[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const float4 g = sphere_geom<kLds>(lds_geom, p, j + k);
                const float ocx = o.x - g.x, ocy = o.y - g.y, ocz = o.z - g.z;
                hb[k] = ocx * d.x + ocy * d.y + ocz * d.z;
                const float cc = (ocx * ocx + ocy * ocy + ocz * ocz) - g.w;
                disc[k] = hb[k] * hb[k] - a * cc;
            }
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                if (!(disc[k] < 0.0f)) {
                    const float sq = __builtin_sqrtf(disc[k]);
                    float root = (-hb[k] - sq) / a;
                    bool ok = true;
                    if (root <= min_t || max_t <= root) {
                        root = (-hb[k] + sq) / a;
                        ok = !(root <= min_t || max_t <= root);
                    }
                    if (ok) {
                        max_t = root;
                        best = j + k;
                    }
                }
            }
        }
        for (; j < n; ++j) {
            const float4 g = sphere_geom<kLds>(lds_geom, p, j);
            const float ocx = o.x - g.x, ocy = o.y - g.y, ocz = o.z - g.z;
            const float hb = ocx * d.x + ocy * d.y + ocz * d.z;
            const float cc = (ocx * ocx + ocy * ocy + ocz * ocz) - g.w;
            const float disc = hb * hb - a * cc;
            if (!(disc < 0.0f)) {
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
        }

        // ---- shade (textures.glsl) or sky (functions.glsl:85-89) ----
        bool ended = false;
        f3 contrib = mk(0.f, 0.f, 0.f);
        if (best >= 0) {
            const float4 g = p.geom[best];
            const float2 rt = p.rt[best];
            const float4 sh = p.shade[best];
            const f3 point = add(scale(max_t, d), o);
            const f3 normal = divs(sub(point, mk(g.x, g.y, g.z)), rt.x);
            const int type = (int)rt.y;
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
            if (sample == p.spp) {
                p.out[out_index] = make_float4(acc.x / spp_f, acc.y / spp_f, acc.z / spp_f, 1.0f);
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
}

}  // namespace

extern "C" __global__ __launch_bounds__(256) void vcrt_trace_lds(TraceParams p) {
    extern __shared__ __attribute__((aligned(16))) float4 lds_geom[];
    trace_impl<true>(p, lds_geom);
}

extern "C" __global__ __launch_bounds__(256) void vcrt_trace_smem(TraceParams p) {
    trace_impl<false>(p, nullptr);
}

// Reassemble the rank-interleaved 16-row stripes gathered from every rank into one frame.
extern "C" __global__ __launch_bounds__(256) void vcrt_assemble(AssembleParams p) {
    const uint32_t total = (uint32_t)p.width * (uint32_t)p.height;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < total;
         i += gridDim.x * blockDim.x) {
        const uint32_t y = i / (uint32_t)p.width, x = i - y * (uint32_t)p.width;
        const uint32_t s = y / (uint32_t)p.stripe_h, within = y - s * (uint32_t)p.stripe_h;
        const uint32_t r = s % (uint32_t)p.world;
        const uint32_t lr = (s / (uint32_t)p.world) * (uint32_t)p.stripe_h + within;
        p.frame[i] =
            p.gathered[((size_t)r * (uint32_t)p.rows_per_rank + lr) * (uint32_t)p.width + x];
    }
}

extern "C" __global__ __launch_bounds__(256) void vcrt_fill(FillParams p) {
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < p.count;
         i += gridDim.x * blockDim.x)
        p.out[i] = p.value;
}
