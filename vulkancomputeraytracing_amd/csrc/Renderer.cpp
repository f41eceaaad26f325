// Renderer.cpp -- the reference's Renderer lifecycle (include/Renderer.hpp:14-20) over the
// C ABI. Begin/Draw/End keep their names, signatures and VkResult convention; the reference's
// compile-time configuration becomes SetRenderDescription / SetRenderScene (optional: without
// them Begin uses the reference defaults of globals.glsl:9-24 and its final scene).
#include <vector>

#include "Renderer.hpp"

namespace {
vcrt_render_desc g_desc;
bool g_desc_set = false;
std::vector<vcrt_sphere> g_scene;
bool g_scene_set = false;
}  // namespace

VkResult SetRenderDescription(IN const vcrt_render_desc* desc) {
    if (!desc) return VK_ERROR_INITIALIZATION_FAILED;
    g_desc = *desc;
    g_desc_set = true;
    return VK_SUCCESS;
}

VkResult SetRenderScene(IN const vcrt_sphere* spheres, IN int32_t count) {
    if (count < 0 || (count > 0 && !spheres)) return VK_ERROR_INITIALIZATION_FAILED;
    g_scene.assign(spheres, spheres + count);
    g_scene_set = true;
    return VK_SUCCESS;
}

// Create pipeline, submit tasks...
VkResult BeginRenderingOperation(void) {
    if (!g_desc_set) vcrt_default_desc(&g_desc);
    VkResult r = vcrt_begin(&g_desc);
    if (r != VK_SUCCESS) return r;
    if (g_scene_set) {
        r = vcrt_set_scene(g_scene.data(), static_cast<int32_t>(g_scene.size()));
        if (r != VK_SUCCESS) {
            vcrt_end();
            return r;
        }
    }
    return VK_SUCCESS;
}

// Draw next frame: one full render, returns when the frame is complete.
VkResult DrawNextFrame(void) { return vcrt_draw_next_frame(); }

// End rendering & destroy allocated environments (idempotent).
VkResult EndRenderingOperation(void) { return vcrt_end(); }

VkResult ReadFramebuffer(OUT float* rgba, IN size_t count) {
    return vcrt_read_framebuffer(rgba, count);
}
