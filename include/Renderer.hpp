/* Renderer.hpp -- the reference's renderer lifecycle (include/Renderer.hpp:14-20) on MI355X.
 *
 * Same three entry points with the same meaning: Begin builds everything the frame loop
 * needs (device buffers, the tracer code object, the scene), DrawNextFrame renders one full
 * frame and returns when it is complete, End tears down and tolerates a partial Begin.
 * The reference's compile-time configuration (globals.glsl:9-24, Common.hpp:23-24) becomes a
 * vcrt_render_desc that may be set before Begin. */
#ifndef VCRT_RENDERER_HPP
#define VCRT_RENDERER_HPP

#include "Common.hpp"

// Create pipeline, submit tasks...
VkResult BeginRenderingOperation(void);

// Draw next frame, to be called by platform handlers (here: the headless frame loop).
VkResult DrawNextFrame(void);

// End rendering & destroy allocated environments.
VkResult EndRenderingOperation(void);

// Additions: configuration and output access (no counterpart in the reference).
VkResult SetRenderDescription(IN const vcrt_render_desc* desc);
VkResult SetRenderScene(IN const vcrt_sphere* spheres, IN int32_t count);
VkResult ReadFramebuffer(OUT float* rgba, IN size_t count);

#endif
