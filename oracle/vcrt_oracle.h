/* vcrt_oracle.h -- CPU restatement of the reference path tracer (TEST INFRASTRUCTURE ONLY).
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this.
 * The product (vulkancomputeraytracing_amd / libvcrt.so) never links or calls it.
 *
 * Restates, quirk for quirk:
 *   shaders/shader.comp:16-58                 (camera block, sample loop, accumulate, store)
 *   shaders/include/functions.glsl:10-92      (rand, hit_sphere, random_in_unit_sphere,
 *                                              modified_refract, schlick, ray_color)
 *   shaders/include/textures.glsl:19-71       (lambertian, glass, metal, dispatcher)
 *   shaders/include/structures.glsl:10-30     (sphere / ray / hit_record layout)
 *   shaders/include/globals.glsl:9-26,29-518  (constants, scene)
 *   SceneGenerator.cpp:10-56                  (mt19937 scene generator)
 */
#ifndef VCRT_ORACLE_H
#define VCRT_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Same field order as GLSL `struct sphere` (structures.glsl:10-16): 40 bytes. */
typedef struct oracle_sphere {
    float center[3];
    float radius;
    float colour[3];
    float texture[3]; /* x = material id (1 lambertian, 2 metal, 3 glass), y = param */
} oracle_sphere;

typedef struct oracle_config {
    int32_t width, height, spp, max_depth;
    float lookfrom[3], lookat[3], vup[3];
    float vfov;
    /* Accumulation (see oracle_render_pixel in vcrt_oracle.c and DESIGN.md section 3). The
     * samples are cut into chunks of accumulate_chunk (0 or >= spp: one chunk), restarting at
     * every progressive frame of frame_spp samples (0: one frame). Each chunk is summed in fp32
     * in sample order. One chunk and no frames: sum / spp in fp32, the reference's sequential
     * sum (shader.comp:46-56) exactly. Otherwise the chunk sums are quantized to 2^-32 and
     * added exactly, then divided in double: the GPU's order-independent combination.
     * accumulate_tail > 0: the last accumulate_tail samples of every frame are cut into chunks
     * of accumulate_tail_chunk instead (the head before them into chunks of accumulate_chunk). */
    int32_t accumulate_chunk;
    int32_t frame_spp;
    int32_t accumulate_tail;
    int32_t accumulate_tail_chunk;
    int32_t accumulate_quantum; /* > 0: runs of this many samples replace the chunk partition */
} oracle_config;

/* Canonical math (see DESIGN.md "canonical math"). */
float oracle_sin(float x);
float oracle_rand(float x, float y);

/* The reference literals the restatement uses, in this order: rand dot x, rand dot y, rand
 * scale (functions.glsl:11), min_t (:76), infinity (globals.glsl:26), sky 0.5 and 1.0
 * (functions.glsl:87), sky bottom 1 and top .5, .7, 1 (:88), jitter offset -0.5
 * (shader.comp:48). */
#define ORACLE_NCONSTANTS 12
void oracle_reference_constants(float out[ORACLE_NCONSTANTS]);

/* shader.comp:18-39 -> out[0..2]=pixel00, [3..5]=delta_u, [6..8]=delta_v, [9..11]=center,
 * [12]=focal_length, [13]=viewport_height, [14]=viewport_width. */
void oracle_camera(const oracle_config* cfg, float out[15]);

/* Render rows y = row_begin, row_begin+row_step, ... < row_end of a W x H frame into rgba
 * (full-frame layout, W*H*4 floats, row 0 = top). Returns 0 on success.
 * segments (optional) receives the number of ray segments (sphere-list scans) traced. */
int oracle_render(const oracle_config* cfg, const oracle_sphere* world, int32_t n,
                  float* rgba, int32_t row_begin, int32_t row_end, int32_t row_step,
                  int32_t threads, uint64_t* segments);

/* The same for a list of pixels: xy = npixels (x, y) pairs, rgba = 4 floats per pixel in list
 * order. Returns 0 on success, -1 on a bad argument (pixel outside the frame). */
int oracle_render_pixels(const oracle_config* cfg, const oracle_sphere* world, int32_t n,
                         const int32_t* xy, int32_t npixels, float* rgba, int32_t threads,
                         uint64_t* segments);

/* The same two renders, with the reference's sequential fp32 sum / spp of every rendered pixel
 * (shader.comp:46-56, one chunk) written to seq_rgba beside the accumulated rgba: one pass. */
int oracle_render_seq(const oracle_config* cfg, const oracle_sphere* world, int32_t n,
                      float* rgba, float* seq_rgba, int32_t row_begin, int32_t row_end,
                      int32_t row_step, int32_t threads, uint64_t* segments);
int oracle_render_pixels_seq(const oracle_config* cfg, const oracle_sphere* world, int32_t n,
                             const int32_t* xy, int32_t npixels, float* rgba, float* seq_rgba,
                             int32_t threads, uint64_t* segments);

/* The quantization scale 2^s of a pixel's quantum sums from the largest |S| among them (all
 * channels, finite sums only): 32 while it is below 2^12, else the largest s with
 * |S| * 2^s < 2^44 (see vcrt_oracle.c). */
int32_t oracle_pixel_scale_log2(float max_abs);

/* Per-pixel radiance of one sample (ray_color), for KATs. */
void oracle_ray_color(const oracle_sphere* world, int32_t n, const float origin[3],
                      const float dir[3], int32_t max_depth, float out[3], uint64_t* segments);

/* Linear rgba32f -> sRGB8 RGBA as a B8G8R8A8_SRGB swapchain stores it (Frontend.cpp:43):
 * channel byte = round-to-nearest of 255 * sRGB(clamp(c,0,1)), NaN -> 0, alpha linear. */
void oracle_encode_srgb8(const float* rgba, size_t pixels, uint8_t* out);

/* SceneGenerator.cpp:23-56 stdout, byte for byte. Returns bytes needed (excl. NUL). */
size_t oracle_scene_generator_text(char* buf, size_t cap);

/* Same generator rules on the square grid [lo,hi)^2, stopping after max_accept accepted
 * spheres (max_accept <= 0: no limit). Values are the "%.2f"-printed decimals parsed as
 * fp32 (the way globals.glsl:31-511 reaches the shader). Returns the count written. */
int32_t oracle_scene_random_spheres(int32_t lo, int32_t hi, int32_t max_accept,
                                    oracle_sphere* out, int32_t cap);

#ifdef __cplusplus
}
#endif
#endif
