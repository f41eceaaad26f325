// vcrt_render -- headless replacement of the reference's main()
// (VulkanComputeRayTracing.cpp:17-42): Begin -> DrawNextFrame x N -> End, then optionally writes
// the frame as PFM (linear rgba32f, as the compute image holds it) or PPM (sRGB8 encoded on the
// GPU, as the B8G8R8A8_SRGB swapchain shows it: Frontend.cpp:43).
#include <cerrno>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "Renderer.hpp"

namespace {

int usage() {
    std::fprintf(stderr,
                 "usage: vcrt_render [--width W] [--height H] [--spp N] [--depth D] "
                 "[--scene final|three|red|stress4096] [--frames F] [--progressive 0|1] [--device I] "
                 "[--out file.ppm|file.pfm]\n");
    return 2;
}

}  // namespace

int main(int argc, char** argv) {
    vcrt_render_desc desc;
    vcrt_default_desc(&desc);
    int scene = VCRT_SCENE_FINAL, frames = 1;
    std::string out;
    bool configured = false;  // any option that changes the description or the scene
    for (int i = 1; i < argc; i++) {
        const std::string a = argv[i];
        if (i + 1 >= argc) return usage();
        const char* v = argv[++i];
        configured = configured || (a != "--out" && a != "--frames");
        if (a == "--width") desc.width = std::atoi(v);
        else if (a == "--height") desc.height = std::atoi(v);
        else if (a == "--spp") desc.samples_per_pixel = std::atoi(v);
        else if (a == "--depth") desc.max_depth = std::atoi(v);
        else if (a == "--frames") frames = std::atoi(v);
        else if (a == "--device") desc.device = std::atoi(v);
        else if (a == "--progressive") desc.progressive = std::atoi(v);
        else if (a == "--out") out = v;
        else if (a == "--scene") {
            const std::string s = v;
            scene = s == "final" ? VCRT_SCENE_FINAL : s == "three" ? VCRT_SCENE_THREE
                  : s == "red" ? VCRT_SCENE_RED : s == "stress4096" ? VCRT_SCENE_STRESS4096 : -1;
            if (scene < 0) return usage();
        } else return usage();
    }
    // Without options this is the reference's main() exactly: Begin/Draw/End with nothing set,
    // so BeginRenderingOperation takes the reference's compile-time configuration (1280x720,
    // 1 spp, depth 50, its camera: globals.glsl:9-24) and its world[] (the final scene).
    if (configured) {
        std::vector<vcrt_sphere> world(8192);
        const int n = vcrt_scene_builtin(scene, world.data(), static_cast<int32_t>(world.size()));
        if (n < 0) return 1;
        world.resize(n);
        SetRenderDescription(&desc);
        SetRenderScene(world.data(), n);
    }
    VkResult r = BeginRenderingOperation();
    if (r != VK_SUCCESS) {
        std::fprintf(stderr, "BeginRenderingOperation: %s\n", vcrt_result_string(r));
        return 1;
    }
    for (int f = 0; f < frames && r == VK_SUCCESS; f++) {
        r = DrawNextFrame();
        vcrt_stats st;
        vcrt_get_stats(&st);
        const double msps = static_cast<double>(st.samples) / (st.frame_ms * 1e3);
        std::printf("frame %d: %s  %.3f ms (kernel %.3f ms)  %.2f Msamples/s  %llu segments\n",
                    f, vcrt_result_string(r), st.frame_ms, st.kernel_ms, msps,
                    static_cast<unsigned long long>(st.segments));
    }
    if (r == VK_SUCCESS && !out.empty()) {
        const bool pfm = out.size() > 4 && out.compare(out.size() - 4, 4, ".pfm") == 0;
        const size_t n = static_cast<size_t>(desc.width) * desc.height;
        std::vector<float> rgba(pfm ? n * 4 : 0);
        std::vector<uint8_t> srgb(pfm ? 0 : n * 4);
        r = pfm ? ReadFramebuffer(rgba.data(), rgba.size())
                : vcrt_read_framebuffer_srgb8(srgb.data(), srgb.size());  // GPU sRGB encode
        FILE* f = r == VK_SUCCESS ? std::fopen(out.c_str(), "wb") : nullptr;
        if (f) {
            std::fprintf(f, pfm ? "PF\n%d %d\n-1.0\n" : "P6\n%d %d\n255\n", desc.width,
                         desc.height);
            for (int y = pfm ? desc.height - 1 : 0; pfm ? y >= 0 : y < desc.height;
                 y += pfm ? -1 : 1) {
                for (int x = 0; x < desc.width; x++) {
                    const size_t i = static_cast<size_t>(y) * desc.width + x;
                    if (pfm) std::fwrite(&rgba[4 * i], sizeof(float), 3, f);
                    else std::fwrite(&srgb[4 * i], 1, 3, f);
                }
            }
            std::fclose(f);
        } else {
            std::fprintf(stderr, "cannot write %s: %s\n", out.c_str(),
                         r == VK_SUCCESS ? std::strerror(errno) : vcrt_result_string(r));
            if (r == VK_SUCCESS) r = VK_ERROR_UNKNOWN;
        }
    }
    EndRenderingOperation();
    return r == VK_SUCCESS ? 0 : 1;
}
