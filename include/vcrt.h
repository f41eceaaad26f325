/* vcrt.h -- C ABI of the MI355X path tracer (libvcrt.so).
 *
 * This is the drop-in boundary. The reference renders from compile-time constants inside one
 * Vulkan compute dispatch; this ABI carries the same state at run time and replaces:
 *
 *   vcrt_begin            <- VkResult BeginRenderingOperation(void)      include/Renderer.hpp:14
 *                            (storage image Renderer.cpp:433-468, compute pipeline :532-543)
 *   vcrt_draw_next_frame  <- VkResult DrawNextFrame(void)                include/Renderer.hpp:17
 *                            (vkCmdDispatch(W/16,H/16,1) Renderer.cpp:221 + submit :678-686)
 *   vcrt_end              <- VkResult EndRenderingOperation(void)        include/Renderer.hpp:20
 *                            (idempotent teardown, tolerates partial Begin: Renderer.cpp:714-774)
 *   vcrt_shader_load      <- VkResult CreateShaderStageFromFile(...)     include/Shader.hpp:14-15
 *                            (loads the gfx950 code object instead of SPIR-V, Shader.cpp:34-95)
 *   vcrt_set_scene        <- const sphere world[]                        globals.glsl:29-518
 *   vcrt_scene_builtin /
 *   vcrt_scene_generator_text <- SceneGenerator executable stdout        SceneGenerator.cpp:23-56
 *   vcrt_render_desc      <- IMAGE_WIDTH/HEIGHT, SAMPLES_PER_PIXEL, MAX_RECURSION_LEVEL, camera
 *                            globals.glsl:9-24, include/Common.hpp:23-24
 *
 * Added (the reference has no equivalents): read-back of the rgba32f framebuffer, statistics,
 * rank/world tile sharding and the tile re-assembly used after a multi-GPU gather.
 *
 * Conventions: plain C types and pointers only. Every function returns a VkResult-compatible
 * int32_t (0 = success, negative = error; values from the Vulkan registry). Nothing throws
 * across the ABI. One renderer per process, calls are not reentrant (as in the reference).
 */
#ifndef VCRT_H
#define VCRT_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef int32_t vcrt_result;

/* VkResult values (Vulkan registry), defined locally: there are no Vulkan headers here. */
#define VCRT_SUCCESS 0
#define VCRT_NOT_READY 1
#define VCRT_ERROR_OUT_OF_HOST_MEMORY (-1)
#define VCRT_ERROR_OUT_OF_DEVICE_MEMORY (-2)
#define VCRT_ERROR_INITIALIZATION_FAILED (-3)
#define VCRT_ERROR_DEVICE_LOST (-4)
#define VCRT_ERROR_FEATURE_NOT_PRESENT (-8)
#define VCRT_ERROR_FORMAT_NOT_SUPPORTED (-11)
#define VCRT_ERROR_UNKNOWN (-13)
#define VCRT_ERROR_INCOMPATIBLE_SHADER_BINARY (1000482000) /* VK_..._SHADER_BINARY_EXT */

/* Material ids, textures.glsl:10-12 */
#define VCRT_TEXTURE_LAMBERTIAN 1
#define VCRT_TEXTURE_METAL 2
#define VCRT_TEXTURE_GLASS 3

/* Same field order and size (40 B) as GLSL `struct sphere`, structures.glsl:10-16. */
typedef struct vcrt_sphere {
    float center[3];
    float radius;
    float colour[3];
    float texture[3]; /* x = material id (as float), y = param (ratio / fuzz / eta), z unused */
} vcrt_sphere;

typedef struct vcrt_camera { /* globals.glsl:21-24 */
    float lookfrom[3];
    float lookat[3];
    float vup[3];
    float vfov; /* degrees */
} vcrt_camera;

/* Kernel variants. SMEM: wave-uniform scalar-cache reads of the linear sphere table (measured
 * faster than LDS staging for 485 and 4100 spheres). CULL: spheres grouped
 * spatially in fours, a group is tested only when some ray of the wave may come near it (same
 * results bit for bit; falls back to SMEM below 16 spheres or for unbounded scenes). AUTO =
 * CULL when it applies, else SMEM. */
#define VCRT_KERNEL_AUTO 0
#define VCRT_KERNEL_LDS 1
#define VCRT_KERNEL_SMEM 2
#define VCRT_KERNEL_CULL 3
#define VCRT_KERNEL_CULL_LANE 4 /* CULL with per-lane group tests (LDS or global tables) */
#define VCRT_KERNEL_CULL_FLAT 5 /* CULL_LANE with the exact tests dealt out over the wave */

typedef struct vcrt_render_desc {
    uint32_t struct_size;      /* sizeof(vcrt_render_desc) */
    int32_t width, height;     /* IMAGE_WIDTH, IMAGE_HEIGHT: each <= 65535; a rank's 8x8 tiles
                                * hold <= 2^26 pixels (8192 x 8192 on one GPU), else vcrt_begin
                                * returns VCRT_ERROR_FORMAT_NOT_SUPPORTED */
    int32_t samples_per_pixel; /* SAMPLES_PER_PIXEL, >= 1 */
    int32_t max_depth;         /* MAX_RECURSION_LEVEL, >= 0 */
    vcrt_camera camera;
    int32_t device;        /* HIP device ordinal; -1 = current device */
    int32_t rank;          /* this process's shard of the frame: the 8x8 tiles (tx, ty) with
                              (tx + ty) % world_size == rank, numbered row-major */
    int32_t world_size;    /* number of shards (GPUs) */
    int32_t kernel_variant;
    int32_t blocks_per_cu; /* persistent grid occupancy; 0 = from the occupancy query */
    int32_t accumulate_chunk; /* samples per work item (0 = 64, halved down to 16 while a pixel
                                 has < 16 items, then while the largest rank's share has
                                 < 2^24 - 2^21 items -- unless the desc takes the cost partition:
                                 chunk and tail left to the rules and a kernel variant with a
                                 cost-order build (AUTO, LDS, SMEM, CULL_FLAT), where the second
                                 halving is skipped, the tail is none and the frames run the cost
                                 order; vcrt_work_chunk), rounded up to a multiple of the quantum
                                 below. A scheduling choice only: it does not change the image. */
    int32_t progressive; /* 0: every DrawNextFrame re-renders samples 0..spp-1 (the reference,
                            Linux.cpp:362-366). 1: frame f renders samples f*spp..(f+1)*spp-1 and
                            the framebuffer holds the average of all frames so far (the same
                            image as one render with (f+1)*spp samples and chunk boundaries at
                            every frame; RENDER_ITERATION, Common.hpp:25, was never wired up). */
    const char* code_object_path; /* NULL = vcrt_tracer.hsaco next to libvcrt.so, then embedded */
    int32_t accumulate_tail;      /* the last accumulate_tail samples of every pixel (of every
                                     progressive frame) in chunks of accumulate_tail_chunk, handed
                                     out after all the other work items, so that the items still
                                     running when the queue drains are short. 0 = the rule
                                     (vcrt_work_tail), -1 = none. Part of the chunk partition: it
                                     schedules only; the image depends on the quantum alone. */
    int32_t accumulate_tail_chunk; /* samples per tail item; 0 = the rule. Tail and tail items
                                      are rounded to multiples of the quantum. */
    int32_t accumulate_quantum; /* the accumulation quantum G (a power of two; 0 = the rule,
                                   vcrt_work_quantum: 4, doubled while a pixel would take more
                                   than 512 quanta). A pixel's samples are summed in fp32 in sample
                                   order within each quantum of G consecutive samples (restarting
                                   at every progressive frame); when one quantum covers the pixel
                                   (G >= samples_per_pixel, not progressive) the sum is divided in
                                   fp32, the reference's sequential sum (shader.comp:46-56)
                                   exactly; otherwise every quantum sum is quantized to 2^-s (s per
                                   pixel from its own quantum sums: vcrt_pixel_scale_log2, 32 for
                                   every pixel of the reference scenes) and added exactly. So the
                                   image depends on G only -- not on the
                                   work items, the schedule or the number of GPUs: a sharded frame
                                   equals a one-GPU render bit for bit. Work items hold whole
                                   quanta. At most 512 quanta per pixel (progressive frames
                                   included). */
} vcrt_render_desc;

typedef struct vcrt_stats {
    uint64_t segments;     /* ray segments traced last frame (one full sphere-list scan each) */
    uint64_t sphere_tests; /* segments * nspheres */
    uint64_t samples;      /* local_rows * width * spp */
    double kernel_ms;      /* tracer kernel time, HIP events on the render stream */
    double frame_ms;       /* host wall time of the last vcrt_draw_next_frame */
    double resolve_ms;     /* resolve kernel time (exact chunk sums -> pixels; 0: one chunk) */
    double gather_ms;      /* multi-GPU frame gather + re-interleave (vcrt_comm_init), HIP events */
    int32_t frames;        /* frames drawn since vcrt_begin */
    int32_t grid_blocks, block_threads, kernel_variant;
    int32_t local_tiles;   /* 8x8 tiles this rank renders */
    int32_t nspheres;
    uint32_t lds_bytes;    /* dynamic LDS of the tracer's tables and stacks (without the ring) */
    int32_t accumulate_chunk; /* samples per work item in effect (head) */
    int32_t tables_in_lds;    /* 1 when the culled scan reads its tables from LDS, 2 when only
                                 its boxes (vcrt_trace_cull_flat_boxes) */
    uint64_t accumulated_spp; /* samples per pixel in the framebuffer (progressive: all frames) */
    uint64_t group_tests;  /* groups of four spheres put through the exact test, per wave */
    uint64_t bound_tests;  /* group bounds tested, per wave (CULL variant) */
    char kernel[48];       /* the tracer kernel the last frame launched (its code-object symbol) */
    uint64_t debug[128]; /* diagnostics (VCRT_DEBUG_STATS=1): [0..7] wave-iterations,
                           active-lane sum, hit groups, fetches, last/first wave end time, sum
                           end time, waves; [8..16] wave clock ticks (s_memtime) in the scan,
                           its uniform levels, node / group / candidate passes (CULL_FLAT),
                           candidate passes run, the whole wave, the big list, node pushes,
                           [17..18] shading and sky, block fetch; [19..22] flat passes:
                           entries dealt, live lanes offered, partial passes, passes; [23]
                           the camera fast trace with its shading; [24..31] camera fast
                           trace entries, its lanes, live lanes, listed-group loop trips and
                           lane sum, root loop trips and lane sum; main-scan hit lanes;
                           [32..39] flat scans: wave ticks in the retire, wave-iterations
                           running the fetch loop, block fetches, items started, next items
                           handed out, item switches in the shading, wave-iterations running
                           the retire, quanta retired (lanes); [40..111] region counters:
                           wave-level entries into the tracer's counted regions (tracer.hip
                           reg::*, in order), summed over the waves */
    int32_t accumulate_tail;       /* tail samples per pixel in effect (0: none) */
    int32_t accumulate_tail_chunk; /* samples per tail item in effect */
    int32_t ring_entries;          /* LDS accumulation ring entries per wave (0: none; the chunk
                                      sums go to global memory directly) */
    int32_t accumulate_quantum;    /* the accumulation quantum G in effect */
    int32_t accumulate_scale_log2; /* the smallest per-pixel quantization scale s of the frame
                                      (vcrt_pixel_scale_log2): 32 unless some pixel's quantum
                                      sums reach 2^12 in magnitude */
    int32_t cost_order;            /* 1: the frame's blocks ran most expensive first (the order
                                      measured by the configuration's first frame; the linear
                                      scans' frames with few items per lane, the cost partition
                                      (accumulate_chunk), or VCRT_WORK_ORDER=cost) */
    int32_t scale_rerenders;       /* renders the last vcrt_draw_next_frame added because a
                                      pixel's quantum sums first reached 2^12 (its scale below 32:
                                      the frame -- progressive: every frame so far -- is rendered
                                      again with each pixel at its own scale) */
} vcrt_stats;

/* Fills *desc with the reference defaults: 1280x720, 1 spp, depth 50, camera
 * (13,2,3)->(0,0,0), vup (0,1,0), vfov 20, rank 0 of 1, stripe 1 (globals.glsl:9-24). */
vcrt_result vcrt_default_desc(vcrt_render_desc* desc);

vcrt_result vcrt_begin(const vcrt_render_desc* desc);
/* The accumulation quantum G that vcrt_begin(desc) uses (the image depends on it alone); host
 * only, no GPU. Negative VkResult for an invalid desc. */
int32_t vcrt_work_quantum(const vcrt_render_desc* desc);
/* Samples per work item of the head that vcrt_begin(desc) uses (a multiple of the quantum);
 * host only, no GPU. Negative VkResult for an invalid desc. */
int32_t vcrt_work_chunk(const vcrt_render_desc* desc);
/* Tail samples per pixel that vcrt_begin(desc) uses (0: none) and, in *tail_chunk, the samples
 * per tail item; host only. The rule: about six head items per lane of the persistent grid,
 * T = 6 * chunk * 327680 / (64 * the largest rank's tiles) rounded to a power of two, in items
 * of max(4, chunk / 8) samples; none when 4 T > samples_per_pixel or chunk >= samples_per_pixel,
 * when the head alone has >= 2 (2^24 - 2^21) items, or for the cost partition (accumulate_chunk).
 * The head ends on a quantum boundary (T is adjusted) and tail items are rounded up to whole
 * quanta. Negative VkResult for an invalid desc. */
int32_t vcrt_work_tail(const vcrt_render_desc* desc, int32_t* tail_chunk);
/* The quantization scale 2^s of a pixel's quantum sums (host only), from E = the largest |S| of
 * its finite quantum sums over every channel (and every progressive frame so far): 32 while
 * E < 2^12 (every pixel of the reference scenes, radiance <= 1 per sample), else the largest s
 * with E * 2^s < 2^44 = 43 - floor(log2 E). Each quantized sum is then an integer below 2^44 and
 * a pixel's (at most 512) of them add exactly in double, whatever the scene's brightness. The
 * renderer measures E while it renders: a frame where some pixel first needs s < 32 is
 * rendered again with every pixel at its own scale (vcrt_stats.scale_rerenders). */
int32_t vcrt_pixel_scale_log2(float max_abs_quantum_sum);
/* Uploads the scene and builds, on the host, its culling tables and the camera-ray lists for
 * this desc's camera and shard (vcrt_cull_tables, vcrt_primary_lists: ~0.1 s for the final
 * scene at 1080p, ~0.4 s for 4100 spheres at 4K). vcrt_begin sets the final scene. */
vcrt_result vcrt_set_scene(const vcrt_sphere* spheres, int32_t count);
vcrt_result vcrt_draw_next_frame(void);
vcrt_result vcrt_end(void);

/* Multi-GPU, one process per GPU (the reference renders on one GPU: Environment.cpp:157-165;
 * "TODO: Cross-GPU sharing", Frontend.cpp:107). Each process calls vcrt_begin with its rank,
 * world_size and device, then vcrt_comm_init with the same id on every rank (rank 0 makes it
 * with vcrt_comm_unique_id and hands it out, e.g. over a TCP store). From then on
 * vcrt_draw_next_frame renders the rank's tiles and gathers every rank's packed tiles to rank 0
 * over RCCL (one grouped send/recv) and re-interleaves them there: on rank 0 it returns with the
 * whole frame, which vcrt_read_framebuffer / vcrt_framebuffer_device then give as [height][width]
 * (the other ranks keep their packed tiles). Collective: every rank must draw every frame.
 * vcrt_end destroys the communicator. */
typedef struct vcrt_comm_id {
    char internal[128]; /* an ncclUniqueId */
} vcrt_comm_id;
vcrt_result vcrt_comm_unique_id(vcrt_comm_id* id);
vcrt_result vcrt_comm_init(const vcrt_comm_id* id);

/* Rank-local framebuffer layout. world_size == 1: the frame, row-major [height][width] (row 0 =
 * top, as the reference's storage image). world_size > 1: packed tiles [tiles][64] with element
 * 8*(y%8) + x%8 of each tile (pixels outside the frame in edge tiles are left untouched). */
vcrt_result vcrt_local_layout(uint32_t* elements, uint32_t* tiles);
/* Copies the rank-local framebuffer (elements * 4 floats, rgba32f) to host memory; count = number
 * of floats available at rgba. */
vcrt_result vcrt_read_framebuffer(float* rgba, size_t count);
/* Device address and size of the framebuffer vcrt_read_framebuffer reads. */
vcrt_result vcrt_framebuffer_device(void** device_ptr, size_t* bytes);
/* Render into caller-owned device memory (>= elements*16 bytes, 16-B aligned); NULL = own.
 * VK_ERROR_FEATURE_NOT_PRESENT after vcrt_comm_init (the gather owns the buffers). */
vcrt_result vcrt_set_framebuffer_device(void* device_ptr, size_t bytes);
/* Rebuild the frame from gathered rank framebuffers: gathered = [world][tiles_per_rank][64]
 * float4 (rank-major, each rank's packed tiles padded to tiles_per_rank), frame = [height][width]
 * float4; both device pointers. Runs on the render stream and returns when done. */
vcrt_result vcrt_assemble_tiles(const void* gathered, void* frame, int32_t width, int32_t height,
                                int32_t world_size, uint32_t tiles_per_rank);
vcrt_result vcrt_get_stats(vcrt_stats* stats);
/* Progressive mode: drop the accumulated frames (sample sequence restarts at 0). */
vcrt_result vcrt_reset_accumulation(void);
/* The rank-local framebuffer encoded as sRGB8 RGBA (alpha linear), as the reference's
 * B8G8R8A8_SRGB swapchain stores it at present time (Frontend.cpp:43; shader.frag:14 copies the
 * texel): channel byte = round-to-nearest of 255 * sRGB(clamp(c, 0, 1)). bytes >= elements*4. */
vcrt_result vcrt_read_framebuffer_srgb8(uint8_t* rgba8, size_t bytes);
/* The 255 ascending linear thresholds behind that encode (byte = #{k : c >= t[k]}). */
void vcrt_srgb8_thresholds(float thresholds[255]);

/* Loads (or reloads) the tracer code object from a file; the analogue of
 * CreateShaderStageFromFile. Returns VCRT_ERROR_INCOMPATIBLE_SHADER_BINARY when the file
 * cannot be read or is not a gfx950 code object. Requires vcrt_begin. */
vcrt_result vcrt_shader_load(const char* filename);

/* Built-in scenes. */
#define VCRT_SCENE_FINAL 0       /* SceneGenerator (481) + big three + ground = 485 spheres */
#define VCRT_SCENE_THREE 1       /* big three + ground (globals.glsl:513-517) = 4 spheres   */
#define VCRT_SCENE_RED 2         /* red Lambertian (0,1,0) r=1 + ground = 2 spheres         */
#define VCRT_SCENE_STRESS4096 3  /* 4096 generated (grid [-33,33)^2) + big three + ground   */
/* Writes up to cap spheres; returns the scene's sphere count, or a negative VkResult. */
int32_t vcrt_scene_builtin(int32_t scene_id, vcrt_sphere* out, int32_t cap);
/* SceneGenerator stdout, byte for byte. Returns the length (excluding NUL); writes up to cap-1
 * bytes plus NUL when buf != NULL. */
size_t vcrt_scene_generator_text(char* buf, size_t cap);

/* The culled scans' grouped tables for a sphere list (host only, no GPU). The big spheres
 * (radius > 8x the median and 5% of the centres' extent) form a short list of groups tested
 * for every ray (*big_groups of them, written first to geom/index); the rest form the
 * hierarchy. Tables: groups of four in pair-SoA form (16 floats each), hierarchy group-pair
 * boxes (16 floats per two groups: lox0 lox1 loy0 loy1 loz0 loz1 hix0 hix1 hiy0 hiy1 hiz0 hiz1
 * K0 K1 0 0 -- the members' extent rounded outwards and K = 8.1u / r_min of the members; a ray
 * rules box i out when its line misses the box grown by its margin, see csrc/tracer.hip
 * box_gap), node-pair boxes (same form; node i covers hierarchy groups 8i..8i+7), top-level
 * boxes (same form; entry i covers hierarchy groups 64i..64i+63, count ceil(G/64) rounded up to
 * even), member indices (4 per group, -1 = padding) and margin4 = {max |centre|, r_max^2, max
 * |box coordinate|, 0} over the hierarchy (rounded up). Returns the hierarchy group count G, a
 * multiple of 16 (0 = culling does not apply: < 16 spheres or unbounded scene), and writes the
 * tables when cap_groups >= *big_groups + G (any pointer may be NULL). */
int32_t vcrt_cull_tables(const vcrt_sphere* spheres, int32_t count, float* geom, float* bound,
                         float* node, float* top, int32_t* index, int32_t* big_groups,
                         float* margin4, int32_t cap_groups);

/* The flat culled scan's camera-ray lists for a scene and render description (host only, no
 * GPU; csrc/primary.cpp): for each 4x4-pixel quarter (qx, qy) of each local tile lt of
 * desc->rank (in the kernels' local-tile order), info[4 lt + 2 qy + qx] = offset << 4 | count
 * of its hierarchy groups in ids (count <= 8), or 15 when it has no list. Returns the number of
 * ids (-1: no culling tables, or an invalid desc), and writes info / ids when cap_tiles (entries
 * of info) / cap_ids are large enough (pointers may be NULL). */
int32_t vcrt_primary_lists(const vcrt_sphere* spheres, int32_t count, const vcrt_render_desc* desc,
                           uint32_t* info, int32_t cap_tiles, uint16_t* ids, int32_t cap_ids);

/* The camera fast trace's per-sphere lists (host only, no GPU; csrc/primary.cpp): for each 4x4
 * quarter as above, info = first pair << 4 | spheres (<= 14), or 15 when it has no list, and the
 * pair records, 12 floats each: (ocx0,ocx1,ocy0,ocy1) (ocz0,ocz1,cc0,cc1) (index0, index1 as
 * int bits, 0, 0), camera-relative as the kernel's exact test computes them (oc = camera centre -
 * centre, cc = |oc|^2 - r^2 in fp32; an odd list pads with oc = 0, cc = 3e38, index -1). Returns
 * the number of pair records (-1: no culling tables, or an invalid desc), and writes info / rec
 * when cap_tiles (entries) / cap_floats are large enough (pointers may be NULL). */
int32_t vcrt_primary_sphere_lists(const vcrt_sphere* spheres, int32_t count,
                                  const vcrt_render_desc* desc, uint32_t* info, int32_t cap_tiles,
                                  float* rec, int32_t cap_floats);

/* Device self-test of the kernel's fast sin path (tracer.hip vcrt_check_sin): for the fp32
 * inputs whose bit patterns are first .. first + count - 1, counts those where the device's
 * sin_fast differs from the canonical sin (must be 0) and those where it fell back to the
 * canonical evaluation, and returns the smallest differing pattern (0xFFFFFFFF if none).
 * Diagnostic addition (the reference has no such call). Requires vcrt_begin. */
vcrt_result vcrt_selftest_sin(uint32_t first, uint32_t count, uint64_t* mismatches,
                              uint64_t* fallbacks, uint32_t* first_mismatch);

/* Canonical math as used by the kernel (host evaluation), for tests and tools. */
float vcrt_canonical_sin(float x);
float vcrt_canonical_rand(float x, float y);

const char* vcrt_result_string(vcrt_result r);

#ifdef __cplusplus
}
#endif
#endif
