// capi.cpp -- the C ABI (include/vcrt.h): renderer state, device buffers, launches.
//
// Replaces the compute half of the reference's Renderer.cpp: the rgba32f storage image
// (Renderer.cpp:433-468) becomes a device float4 buffer, the compute pipeline
// (:532-543) a HIP module, and the per-frame vkCmdDispatch(W/16,H/16,1) + vkQueueSubmit
// (:204-225, :673-686) one persistent-kernel launch on a HIP stream. All state is file-static,
// as in the reference (Renderer.cpp:13-33): one renderer per process.
#include <dlfcn.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include <hip/hip_runtime_api.h>

#include "Shader.hpp"
#include "hip_status.hpp"
#include "scene.hpp"
#include "vcrt.h"
#include "vcrt_kernel_abi.h"
#include "vcrt_math.h"

namespace {

using vcrt::to_vk;

constexpr size_t kCounterBytes = 256;  // work counter (u32) + segment counter (u64), padded

struct RendererState {
    bool begun = false;
    vcrt_render_desc desc{};
    int device = 0;
    int num_cus = 0;
    size_t max_lds = 0;
    hipStream_t stream = nullptr;
    hipEvent_t ev_start = nullptr, ev_stop = nullptr;
    VkPipelineShaderStageCreateInfo stage{};
    hipFunction_t k_trace_lds = nullptr, k_trace_smem = nullptr, k_assemble = nullptr,
                  k_fill = nullptr;
    // scene
    int32_t nspheres = 0;
    float4* d_geom = nullptr;
    float4* d_shade = nullptr;
    float2* d_rt = nullptr;
    // per-frame inputs / outputs
    float2* d_jitter = nullptr;
    float4* d_fb_own = nullptr;
    float4* d_fb = nullptr;  // current render target (own or caller-provided)
    size_t fb_bytes = 0;
    void* d_counters = nullptr;
    int32_t local_rows = 0;
    vcrt::Camera cam{};
    vcrt_stats stats{};
};

RendererState g;

#define VCRT_TRY(expr)                          \
    do {                                        \
        hipError_t e_ = (expr);                 \
        if (e_ != hipSuccess) return to_vk(e_); \
    } while (0)

int32_t rows_for_rank(int32_t height, int32_t stripe, int32_t world, int32_t rank) {
    int32_t rows = 0;
    for (int32_t s = rank; s * stripe < height; s += world)
        rows += std::min(stripe, height - s * stripe);
    return rows;
}

// Directory of this shared object (for the default code-object path).
std::string library_dir() {
    Dl_info info;
    if (dladdr(reinterpret_cast<void*>(&rows_for_rank), &info) && info.dli_fname) {
        std::string p(info.dli_fname);
        const size_t slash = p.find_last_of('/');
        if (slash != std::string::npos) return p.substr(0, slash);
    }
    return ".";
}

void free_scene() {
    if (g.d_geom) (void)hipFree(g.d_geom);
    if (g.d_shade) (void)hipFree(g.d_shade);
    if (g.d_rt) (void)hipFree(g.d_rt);
    g.d_geom = nullptr;
    g.d_shade = nullptr;
    g.d_rt = nullptr;
    g.nspheres = 0;
}

VkResult bind_kernels() {
    hipModule_t m = static_cast<hipModule_t>(g.stage.module);
    VCRT_TRY(hipModuleGetFunction(&g.k_trace_lds, m, "vcrt_trace_lds"));
    VCRT_TRY(hipModuleGetFunction(&g.k_trace_smem, m, "vcrt_trace_smem"));
    VCRT_TRY(hipModuleGetFunction(&g.k_assemble, m, "vcrt_assemble"));
    VCRT_TRY(hipModuleGetFunction(&g.k_fill, m, "vcrt_fill"));
    return VK_SUCCESS;
}

VkResult load_code_object(const char* path) {
    VkPipelineShaderStageCreateInfo stage{};
    VkResult r;
    if (path) {
        r = CreateShaderStageFromFile(path, VK_SHADER_STAGE_COMPUTE_BIT, &stage);
    } else {
        const std::string def = library_dir() + "/vcrt_tracer.hsaco";
        r = access(def.c_str(), R_OK) == 0
                ? CreateShaderStageFromFile(def.c_str(), VK_SHADER_STAGE_COMPUTE_BIT, &stage)
                : VK_ERROR_INCOMPATIBLE_SHADER_BINARY_EXT;
        if (r != VK_SUCCESS)  // embedded copy, as LOAD_SHADER_FROM_MEMORY
            r = CreateShaderStageFromFile(nullptr, VK_SHADER_STAGE_COMPUTE_BIT, &stage);
    }
    if (r != VK_SUCCESS) return r;
    DestroyShaderStage(&g.stage);
    g.stage = stage;
    return bind_kernels();
}

bool desc_valid(const vcrt_render_desc& d) {
    if (d.struct_size != sizeof(vcrt_render_desc)) return false;
    if (d.width <= 0 || d.height <= 0 || d.samples_per_pixel <= 0 || d.max_depth < 0)
        return false;
    if (static_cast<int64_t>(d.width) * d.height > (int64_t{1} << 31)) return false;
    if (d.world_size <= 0 || d.rank < 0 || d.rank >= d.world_size) return false;
    if (d.stripe_height < 0 || d.blocks_per_cu < 0) return false;
    if (d.kernel_variant < VCRT_KERNEL_AUTO || d.kernel_variant > VCRT_KERNEL_SMEM) return false;
    return true;
}

template <typename Params>
VkResult launch(hipFunction_t f, uint32_t grid, uint32_t block, uint32_t lds, Params& params) {
    void* args[] = {&params};
    VCRT_TRY(hipModuleLaunchKernel(f, grid, 1, 1, block, 1, 1, lds, g.stream, args, nullptr));
    return VK_SUCCESS;
}

}  // namespace

extern "C" {

vcrt_result vcrt_default_desc(vcrt_render_desc* d) {
    if (!d) return VCRT_ERROR_INITIALIZATION_FAILED;
    std::memset(d, 0, sizeof(*d));
    d->struct_size = sizeof(vcrt_render_desc);
    d->width = 1280;  // globals.glsl:16-17
    d->height = 720;
    d->samples_per_pixel = 1;  // globals.glsl:9-13 (#if 0 -> 1)
    d->max_depth = 50;         // globals.glsl:14
    const float from[3] = {13, 2, 3}, at[3] = {0, 0, 0}, up[3] = {0, 1, 0};
    std::memcpy(d->camera.lookfrom, from, sizeof(from));
    std::memcpy(d->camera.lookat, at, sizeof(at));
    std::memcpy(d->camera.vup, up, sizeof(up));
    d->camera.vfov = 20.0f;
    d->device = -1;
    d->rank = 0;
    d->world_size = 1;
    d->stripe_height = 16;
    d->kernel_variant = VCRT_KERNEL_AUTO;
    return VCRT_SUCCESS;
}

vcrt_result vcrt_begin(const vcrt_render_desc* desc) {
    if (!desc || !desc_valid(*desc)) return VCRT_ERROR_INITIALIZATION_FAILED;
    if (g.begun) vcrt_end();
    g = RendererState{};
    g.desc = *desc;
    if (g.desc.stripe_height == 0) g.desc.stripe_height = 16;
    g.begun = true;  // from here on vcrt_end() cleans up whatever was created

    int count = 0;
    hipError_t e = hipGetDeviceCount(&count);
    if (e != hipSuccess || count == 0) {
        vcrt_end();
        return VCRT_ERROR_INITIALIZATION_FAILED;
    }
    if (g.desc.device >= 0) {
        if (g.desc.device >= count || hipSetDevice(g.desc.device) != hipSuccess) {
            vcrt_end();
            return VCRT_ERROR_INITIALIZATION_FAILED;
        }
    }
    VkResult r = VK_SUCCESS;
    auto fail = [&](VkResult rr) {
        vcrt_end();
        return rr;
    };
    if ((r = to_vk(hipGetDevice(&g.device))) != VK_SUCCESS) return fail(r);
    hipDeviceProp_t prop;
    if ((r = to_vk(hipGetDeviceProperties(&prop, g.device))) != VK_SUCCESS) return fail(r);
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
        return fail(VCRT_ERROR_FEATURE_NOT_PRESENT);  // code object is gfx950-only
    g.num_cus = prop.multiProcessorCount;
    g.max_lds = prop.sharedMemPerBlock;
    if ((r = to_vk(hipStreamCreateWithFlags(&g.stream, hipStreamNonBlocking))) != VK_SUCCESS)
        return fail(r);
    if ((r = to_vk(hipEventCreate(&g.ev_start))) != VK_SUCCESS) return fail(r);
    if ((r = to_vk(hipEventCreate(&g.ev_stop))) != VK_SUCCESS) return fail(r);
    if ((r = load_code_object(g.desc.code_object_path)) != VK_SUCCESS) return fail(r);
    g.desc.code_object_path = nullptr;  // not owned

    // Camera (shader.comp:18-39): uniform per dispatch, computed once here.
    const vcrt_camera& c = g.desc.camera;
    g.cam = vcrt::make_camera(g.desc.width, g.desc.height,
                              vcrt::mk(c.lookfrom[0], c.lookfrom[1], c.lookfrom[2]),
                              vcrt::mk(c.lookat[0], c.lookat[1], c.lookat[2]),
                              vcrt::mk(c.vup[0], c.vup[1], c.vup[2]), c.vfov,
                              [](double x) { return std::tan(x); });
    // Jitter (shader.comp:48) depends only on the sample index: one table per frame config.
    const int spp = g.desc.samples_per_pixel;
    std::vector<float2> jitter(static_cast<size_t>(spp));
    for (int i = 0; i < spp; i++) {
        jitter[i].x = -0.5f + vcrt::rand2(static_cast<float>(i), static_cast<float>(i));
        jitter[i].y = -0.5f + vcrt::rand2(static_cast<float>(i + 1), static_cast<float>(i + 1));
    }
    if ((r = to_vk(hipMalloc(&g.d_jitter, sizeof(float2) * spp))) != VK_SUCCESS) return fail(r);
    if ((r = to_vk(hipMemcpy(g.d_jitter, jitter.data(), sizeof(float2) * spp,
                             hipMemcpyHostToDevice))) != VK_SUCCESS)
        return fail(r);

    g.local_rows = rows_for_rank(g.desc.height, g.desc.stripe_height, g.desc.world_size,
                                 g.desc.rank);
    g.fb_bytes = static_cast<size_t>(g.local_rows) * g.desc.width * sizeof(float4);
    if (g.fb_bytes) {
        if ((r = to_vk(hipMalloc(&g.d_fb_own, g.fb_bytes))) != VK_SUCCESS) return fail(r);
        if ((r = to_vk(hipMemset(g.d_fb_own, 0, g.fb_bytes))) != VK_SUCCESS) return fail(r);
    }
    g.d_fb = g.d_fb_own;
    if ((r = to_vk(hipMalloc(&g.d_counters, kCounterBytes))) != VK_SUCCESS) return fail(r);

    // The reference's world[] is compiled in; default to the same final scene.
    std::vector<vcrt_sphere> world;
    vcrt::builtin_scene(VCRT_SCENE_FINAL, world);
    if ((r = vcrt_set_scene(world.data(), static_cast<int32_t>(world.size()))) != VK_SUCCESS)
        return fail(r);
    g.stats.local_rows = g.local_rows;
    return VCRT_SUCCESS;
}

vcrt_result vcrt_set_scene(const vcrt_sphere* spheres, int32_t count) {
    if (!g.begun) return VCRT_ERROR_INITIALIZATION_FAILED;
    if (count < 0 || (count > 0 && !spheres)) return VCRT_ERROR_INITIALIZATION_FAILED;
    std::vector<float4> geom(count), shade(count);
    std::vector<float2> rt(count);
    for (int32_t i = 0; i < count; i++) {
        const vcrt_sphere& s = spheres[i];
        const float r2 = s.radius * s.radius;  // s.radius*s.radius, functions.glsl:18
        geom[i] = make_float4(s.center[0], s.center[1], s.center[2], r2);
        shade[i] = make_float4(s.colour[0], s.colour[1], s.colour[2], s.texture[1]);
        rt[i] = make_float2(s.radius, s.texture[0]);
    }
    (void)hipStreamSynchronize(g.stream);
    free_scene();
    if (count > 0) {
        VCRT_TRY(hipMalloc(&g.d_geom, sizeof(float4) * count));
        VCRT_TRY(hipMalloc(&g.d_shade, sizeof(float4) * count));
        VCRT_TRY(hipMalloc(&g.d_rt, sizeof(float2) * count));
        VCRT_TRY(hipMemcpy(g.d_geom, geom.data(), sizeof(float4) * count, hipMemcpyHostToDevice));
        VCRT_TRY(
            hipMemcpy(g.d_shade, shade.data(), sizeof(float4) * count, hipMemcpyHostToDevice));
        VCRT_TRY(hipMemcpy(g.d_rt, rt.data(), sizeof(float2) * count, hipMemcpyHostToDevice));
    }
    g.nspheres = count;
    g.stats.nspheres = count;
    return VCRT_SUCCESS;
}

vcrt_result vcrt_draw_next_frame(void) {
    if (!g.begun || !g.stage.module) return VCRT_ERROR_INITIALIZATION_FAILED;
    const auto t0 = std::chrono::steady_clock::now();
    const uint32_t items = static_cast<uint32_t>(g.local_rows) * g.desc.width;
    g.stats.segments = 0;
    g.stats.kernel_ms = 0.0;
    if (items != 0 && g.desc.max_depth == 0) {
        // ray_color with MAX_RECURSION_LEVEL 0 returns its undefined value (canonical 0) for
        // every sample without scanning: the frame is (0,0,0,1).
        vcrt::FillParams fp{g.d_fb, items, make_float4(0.f, 0.f, 0.f, 1.f)};
        const uint32_t grid = std::min<uint32_t>((items + 255) / 256, 4096);
        VkResult r = launch(g.k_fill, grid, 256, 0, fp);
        if (r != VK_SUCCESS) return r;
    }
    if (items != 0 && g.desc.max_depth > 0) {
        vcrt::TraceParams p{};
        p.geom = g.d_geom;
        p.shade = g.d_shade;
        p.rt = g.d_rt;
        p.jitter = g.d_jitter;
        p.out = g.d_fb;
        p.work = static_cast<uint32_t*>(g.d_counters);
        p.segments = reinterpret_cast<unsigned long long*>(static_cast<char*>(g.d_counters) + 8);
        p.nspheres = g.nspheres;
        p.width = g.desc.width;
        p.height = g.desc.height;
        p.spp = g.desc.samples_per_pixel;
        p.max_depth = g.desc.max_depth;
        p.rank = g.desc.rank;
        p.world = g.desc.world_size;
        p.stripe_h = g.desc.stripe_height;
        p.local_rows = g.local_rows;
        p.total_items = items;
        const vcrt::f3 v[4] = {g.cam.pixel00, g.cam.delta_u, g.cam.delta_v, g.cam.center};
        for (int i = 0; i < 4; i++) {
            p.cam[3 * i + 0] = v[i].x;
            p.cam[3 * i + 1] = v[i].y;
            p.cam[3 * i + 2] = v[i].z;
        }
        const uint32_t geom_lds = static_cast<uint32_t>(sizeof(float4) * g.nspheres);
        int variant = g.desc.kernel_variant;
        if (variant == VCRT_KERNEL_AUTO)
            variant = geom_lds <= 40 * 1024 ? VCRT_KERNEL_LDS : VCRT_KERNEL_SMEM;
        if (variant == VCRT_KERNEL_LDS && geom_lds > g.max_lds) variant = VCRT_KERNEL_SMEM;
        hipFunction_t f = variant == VCRT_KERNEL_LDS ? g.k_trace_lds : g.k_trace_smem;
        const uint32_t lds = variant == VCRT_KERNEL_LDS ? geom_lds : 0;
        const uint32_t block = 256;
        int per_cu = g.desc.blocks_per_cu;
        if (per_cu <= 0) {
            per_cu = 0;
            if (hipModuleOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, f, block, lds) !=
                    hipSuccess ||
                per_cu <= 0)
                per_cu = 1;
        }
        const uint32_t grid = static_cast<uint32_t>(per_cu) * static_cast<uint32_t>(g.num_cus);
        VCRT_TRY(hipMemsetAsync(g.d_counters, 0, kCounterBytes, g.stream));
        VCRT_TRY(hipEventRecord(g.ev_start, g.stream));
        VkResult r = launch(f, grid, block, lds, p);
        if (r != VK_SUCCESS) return r;
        VCRT_TRY(hipEventRecord(g.ev_stop, g.stream));
        unsigned long long counters[2] = {0, 0};
        VCRT_TRY(hipMemcpyAsync(counters, g.d_counters, sizeof(counters), hipMemcpyDeviceToHost,
                                g.stream));
        VCRT_TRY(hipStreamSynchronize(g.stream));
        float ms = 0.f;
        VCRT_TRY(hipEventElapsedTime(&ms, g.ev_start, g.ev_stop));
        g.stats.kernel_ms = ms;
        g.stats.segments = counters[1];
        g.stats.grid_blocks = static_cast<int32_t>(grid);
        g.stats.block_threads = static_cast<int32_t>(block);
        g.stats.kernel_variant = variant;
        g.stats.lds_bytes = lds;
    }
    VCRT_TRY(hipStreamSynchronize(g.stream));
    g.stats.sphere_tests = g.stats.segments * static_cast<uint64_t>(g.nspheres);
    g.stats.samples =
        static_cast<uint64_t>(items) * static_cast<uint64_t>(g.desc.samples_per_pixel);
    g.stats.frames += 1;
    g.stats.frame_ms =
        std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    return VCRT_SUCCESS;
}

vcrt_result vcrt_end(void) {
    if (!g.begun) return VCRT_SUCCESS;  // idempotent
    if (g.stream) (void)hipStreamSynchronize(g.stream);
    free_scene();
    if (g.d_jitter) (void)hipFree(g.d_jitter);
    if (g.d_fb_own) (void)hipFree(g.d_fb_own);
    if (g.d_counters) (void)hipFree(g.d_counters);
    DestroyShaderStage(&g.stage);
    if (g.ev_start) (void)hipEventDestroy(g.ev_start);
    if (g.ev_stop) (void)hipEventDestroy(g.ev_stop);
    if (g.stream) (void)hipStreamDestroy(g.stream);
    g = RendererState{};
    return VCRT_SUCCESS;
}

vcrt_result vcrt_local_rows(int32_t* rows) {
    if (!g.begun || !rows) return VCRT_ERROR_INITIALIZATION_FAILED;
    *rows = g.local_rows;
    return VCRT_SUCCESS;
}

vcrt_result vcrt_read_framebuffer(float* rgba, size_t count) {
    if (!g.begun || (!rgba && g.fb_bytes)) return VCRT_ERROR_INITIALIZATION_FAILED;
    if (count * sizeof(float) < g.fb_bytes) return VCRT_ERROR_FORMAT_NOT_SUPPORTED;
    if (g.fb_bytes) VCRT_TRY(hipMemcpy(rgba, g.d_fb, g.fb_bytes, hipMemcpyDeviceToHost));
    return VCRT_SUCCESS;
}

vcrt_result vcrt_framebuffer_device(void** device_ptr, size_t* bytes) {
    if (!g.begun || !device_ptr || !bytes) return VCRT_ERROR_INITIALIZATION_FAILED;
    *device_ptr = g.d_fb;
    *bytes = g.fb_bytes;
    return VCRT_SUCCESS;
}

vcrt_result vcrt_set_framebuffer_device(void* device_ptr, size_t bytes) {
    if (!g.begun) return VCRT_ERROR_INITIALIZATION_FAILED;
    if (device_ptr == nullptr) {
        g.d_fb = g.d_fb_own;
        return VCRT_SUCCESS;
    }
    if (bytes < g.fb_bytes || (reinterpret_cast<uintptr_t>(device_ptr) & 15u))
        return VCRT_ERROR_FORMAT_NOT_SUPPORTED;
    g.d_fb = static_cast<float4*>(device_ptr);
    return VCRT_SUCCESS;
}

vcrt_result vcrt_assemble_stripes(const void* gathered, void* frame, int32_t width,
                                  int32_t height, int32_t world_size, int32_t stripe_height,
                                  int32_t rows_per_rank) {
    if (!g.begun || !gathered || !frame) return VCRT_ERROR_INITIALIZATION_FAILED;
    if (width <= 0 || height <= 0 || world_size <= 0 || stripe_height <= 0)
        return VCRT_ERROR_INITIALIZATION_FAILED;
    for (int32_t r = 0; r < world_size; r++)
        if (rows_for_rank(height, stripe_height, world_size, r) > rows_per_rank)
            return VCRT_ERROR_FORMAT_NOT_SUPPORTED;
    vcrt::AssembleParams ap{static_cast<const float4*>(gathered), static_cast<float4*>(frame),
                            width, height, world_size, stripe_height, rows_per_rank};
    const uint64_t total = static_cast<uint64_t>(width) * height;
    const uint32_t grid = static_cast<uint32_t>(std::min<uint64_t>((total + 255) / 256, 8192));
    VkResult r = launch(g.k_assemble, grid, 256, 0, ap);
    if (r != VK_SUCCESS) return r;
    VCRT_TRY(hipStreamSynchronize(g.stream));
    return VCRT_SUCCESS;
}

vcrt_result vcrt_get_stats(vcrt_stats* stats) {
    if (!g.begun || !stats) return VCRT_ERROR_INITIALIZATION_FAILED;
    *stats = g.stats;
    return VCRT_SUCCESS;
}

vcrt_result vcrt_shader_load(const char* filename) {
    if (!g.begun) return VCRT_ERROR_INITIALIZATION_FAILED;
    if (!filename) return VCRT_ERROR_INCOMPATIBLE_SHADER_BINARY;
    (void)hipStreamSynchronize(g.stream);
    return load_code_object(filename);
}

int32_t vcrt_scene_builtin(int32_t scene_id, vcrt_sphere* out, int32_t cap) {
    std::vector<vcrt_sphere> s;
    const int r = vcrt::builtin_scene(scene_id, s);
    if (r != VCRT_SUCCESS) return r;
    if (out)
        std::copy_n(s.begin(), std::min<size_t>(s.size(), static_cast<size_t>(std::max(cap, 0))),
                    out);
    return static_cast<int32_t>(s.size());
}

size_t vcrt_scene_generator_text(char* buf, size_t cap) {
    const std::string t = vcrt::scene_generator_text();
    if (buf && cap) {
        const size_t k = std::min(t.size(), cap - 1);
        std::memcpy(buf, t.data(), k);
        buf[k] = '\0';
    }
    return t.size();
}

float vcrt_canonical_sin(float x) { return vcrt::sin_canonical(x); }
float vcrt_canonical_rand(float x, float y) { return vcrt::rand2(x, y); }

const char* vcrt_result_string(vcrt_result r) {
    switch (r) {
        case VCRT_SUCCESS: return "VK_SUCCESS";
        case VCRT_NOT_READY: return "VK_NOT_READY";
        case VCRT_ERROR_OUT_OF_HOST_MEMORY: return "VK_ERROR_OUT_OF_HOST_MEMORY";
        case VCRT_ERROR_OUT_OF_DEVICE_MEMORY: return "VK_ERROR_OUT_OF_DEVICE_MEMORY";
        case VCRT_ERROR_INITIALIZATION_FAILED: return "VK_ERROR_INITIALIZATION_FAILED";
        case VCRT_ERROR_DEVICE_LOST: return "VK_ERROR_DEVICE_LOST";
        case VCRT_ERROR_FEATURE_NOT_PRESENT: return "VK_ERROR_FEATURE_NOT_PRESENT";
        case VCRT_ERROR_FORMAT_NOT_SUPPORTED: return "VK_ERROR_FORMAT_NOT_SUPPORTED";
        case VCRT_ERROR_UNKNOWN: return "VK_ERROR_UNKNOWN";
        case VCRT_ERROR_INCOMPATIBLE_SHADER_BINARY: return "VK_ERROR_INCOMPATIBLE_SHADER_BINARY_EXT";
        default: return "VK_RESULT_UNRECOGNIZED";
    }
}

}  // extern "C"
