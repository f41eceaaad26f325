// vcrt_kernel_abi.h -- argument blocks passed by value to the gfx950 kernels of
// vcrt_tracer.hsaco (host: capi.cpp via hipModuleLaunchKernel; device: tracer.hip).
#pragma once

#include <cstdint>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#else
#include <hip/hip_runtime_api.h>
#include <hip/hip_vector_types.h>
#endif

namespace vcrt {

// Work items are (8x8 tile, sample chunk, lane slot): 64 consecutive items are one tile of
// pixels at one chunk of samples (see tracer.hip). Pixels q = 0..total_pixels-1 are numbered
// in 8-row bands with eight rows of one column per 8 consecutive q.
struct TraceParams {
    const float4* geom;           // pair-SoA sphere groups (+1 padding group), scan input
    const float4* center_radius;  // [n] (center.xyz, radius)           -- read once per hit
    const float4* shade;          // [n] (colour.rgb, texture.y = param)
    const float* material;        // [n] texture.x = material id
    const float2* jitter;  // [spp] (-0.5+rand(i,i), -0.5+rand(i+1,i+1)), shader.comp:48
    float4* out;           // [local_rows * width] rank-local framebuffer, rgba32f
    float4* partial;       // [nchunks][total_pixels] chunk sums (nchunks > 1)
    uint32_t* work;        // work-item counter, zeroed before every launch
    unsigned long long* segments;  // ray segments traced, zeroed before every launch
    unsigned long long* debug;     // diagnostics counters (stats kernels only), may be null
    int32_t nspheres;
    int32_t width, height, spp, max_depth;
    int32_t rank, world, stripe_h, local_rows;
    uint32_t total_pixels;  // local_rows * width
    uint32_t total_items;   // ceil(total_pixels / 64) * 64 * nchunks
    int32_t chunk;          // samples per work item
    int32_t nchunks;        // ceil(spp / chunk)
    uint32_t flags;         // kFlag*
    float cam[12];          // pixel00.xyz, delta_u.xyz, delta_v.xyz, center.xyz
};

constexpr uint32_t kFlagReverseOrder = 1u;  // hand out work items last-to-first

struct ResolveParams {
    const float4* partial;  // [nchunks][total_pixels]
    float4* out;            // [local_rows * width]
    uint32_t total_pixels;
    int32_t nchunks, spp, width, local_rows;
};

struct AssembleParams {
    const float4* gathered;  // [world][rows_per_rank][width] packed rank framebuffers
    float4* frame;           // [height][width]
    int32_t width, height, world, stripe_h, rows_per_rank;
};

struct FillParams {
    float4* out;
    uint32_t count;
    float4 value;
};

}  // namespace vcrt
