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

// Work items are the rank's pixels in 8-row bands, 8 rows x 1 column per 8 consecutive
// items, so 64 consecutive items form an 8x8 tile (see item_to_pixel in tracer.hip).
struct TraceParams {
    const float4* geom;   // [n] (center.xyz, radius*radius)      -- hot: read every segment
    const float4* shade;  // [n] (colour.rgb, texture.y = param)  -- read once per hit
    const float2* rt;     // [n] (radius, texture.x = material id)
    const float2* jitter; // [spp] (-0.5+rand(i,i), -0.5+rand(i+1,i+1)), shader.comp:48
    float4* out;          // [local_rows * width] rank-local framebuffer, rgba32f
    uint32_t* work;       // pixel work counter, zeroed before every launch
    unsigned long long* segments;  // ray segments traced, zeroed before every launch
    int32_t nspheres;
    int32_t width, height, spp, max_depth;
    int32_t rank, world, stripe_h, local_rows;
    uint32_t total_items;  // local_rows * width
    float cam[12];         // pixel00.xyz, delta_u.xyz, delta_v.xyz, center.xyz
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
