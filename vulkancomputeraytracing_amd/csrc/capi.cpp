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
#include <array>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <utility>
#include <vector>

#include <hip/hip_runtime_api.h>
#include <rccl/rccl.h>

#include "Shader.hpp"
#include "cluster.hpp"
#include "comm_wait.hpp"
#include "hip_status.hpp"
#include "scene.hpp"
#include "vcrt.h"
#include "vcrt_kernel_abi.h"
#include "vcrt_math.h"

namespace {

using vcrt::to_vk;

// segments (u64 at 8), work_done[2] (u64 at 16), then the work-queue counters from 256
constexpr size_t kCounterBytes = 256 + vcrt::kMaxQueues * 4 * vcrt::kQueueStride;
// LDS for the SMEM scan's staged tables (a few spheres' shading rows and the jitter table)
constexpr uint32_t kStageMaxBytes = 8192;
constexpr int32_t kDefaultChunk = 64;        // samples per work item (upper end)
constexpr uint32_t kRegionCount = 88;       // tracer.hip kRegions: region counters per wave
constexpr uint32_t kRegionDebugBase = 40;   // their sums in vcrt_stats.debug[40..127]

struct RendererState {
    bool begun = false;
    vcrt_render_desc desc{};
    int device = 0;
    int num_cus = 0;
    size_t max_lds = 0;
    hipStream_t stream = nullptr;
    hipEvent_t ev_start = nullptr, ev_stop = nullptr, ev_resolve = nullptr;
    VkPipelineShaderStageCreateInfo stage{};
    hipFunction_t k_trace_lds = nullptr, k_trace_smem = nullptr, k_assemble = nullptr,
                  k_fill = nullptr, k_trace_lds_stats = nullptr, k_trace_smem_stats = nullptr,
                  k_resolve = nullptr, k_encode = nullptr, k_trace_cull = nullptr,
                  k_trace_cull_stats = nullptr, k_trace_cull_lane_lds = nullptr,
                  k_trace_cull_lane_lds_stats = nullptr, k_trace_cull_lane = nullptr,
                  k_trace_cull_lane_stats = nullptr, k_trace_cull_lane_lds_wide = nullptr,
                  k_trace_cull_lane_lds_wide_stats = nullptr, k_trace_cull_flat = nullptr,
                  k_trace_cull_flat_stats = nullptr, k_trace_cull_flat_global = nullptr,
                  k_trace_cull_flat_global_stats = nullptr, k_trace_cull_flat_boxes = nullptr,
                  k_trace_cull_flat_boxes_stats = nullptr, k_setup_jitter = nullptr;
    // the flat scans' cost-order builds (null: the code object predates them; no cost order)
    hipFunction_t k_trace_cull_flat_cost = nullptr, k_trace_cull_flat_global_cost = nullptr,
                  k_trace_cull_flat_boxes_cost = nullptr;
    // VCRT_CULL_LANE_TABLES: 0 = auto, 1 = LDS, 2 = global, 3 = boxes in LDS (flat scan)
    int cull_lane_tables = 0;
    bool accum_ring = true;      // VCRT_ACCUM_RING=0: chunk sums straight to global memory
    bool stage_tables = true;    // VCRT_STAGE_TABLES=0: the SMEM scan reads its tables globally
    uint32_t ring_max = vcrt::kRingMaxEntries;
    int max_blocks_per_cu = 0;  // VCRT_MAX_BLOCKS_PER_CU: caps the occupancy rule (0: none)
    // the cost-ordered schedule ("cost order" in vcrt_draw_next_frame): -1 auto, 0 off, 1 on
    // (VCRT_WORK_ORDER=cost / static); the first frame of a configuration measures each pixel's
    // segments, later frames hand out the blocks most expensive first
    int cost_order = -1;
    bool cost_partition = false;  // the partition is the cost partition (default_chunk)
    uint32_t* d_pixel_cost = nullptr;   // [total_pixels] segments (TraceParams.pixel_cost)
    uint32_t* d_block_order = nullptr;  // [blocks] TraceParams.block_order
    size_t cost_words = 0, order_words = 0;
    uint64_t order_key = 0;  // the configuration the order was measured for (0: none)
    uint32_t nch_magic[2] = {0u, 0u};  // TraceParams.nch_magic of the partition
    // deferred fetches (TraceParams.fetch_min / fetch_wait; VCRT_FETCH_MIN, VCRT_FETCH_WAIT;
    // fetch_min 0: the rule in trace_frame)
    uint32_t fetch_min = 0u, fetch_wait = 0u;
    int flat_block = 0;  // VCRT_FLAT_BLOCK: threads per group of the LDS flat scan (0: 256)
    uint32_t lds_per_cu = 0;     // LDS bytes per CU (160 KB on gfx950)
    // diagnostics (environment: VCRT_DEBUG_STATS=1, VCRT_WORK_ORDER=forward)
    int debug_stats = 0;  // 1: the stats kernels; 2: the product kernels with a debug buffer
                          //    (builds with VCRT_WAVE_END_TIMES record wave start/end times)
    uint32_t work_flags = 0;
    void* d_debug = nullptr;
    uint32_t* d_region = nullptr;  // stats kernels: [waves][kRegionCount] region entry counts
    size_t region_words = 0;
    // scene
    int32_t nspheres = 0;
    bool scene_bounded = false;  // every |center|, radius <= 2^30: discriminants stay finite
    bool radii_safe = false;     // every |radius| in [2^-40, 2^30] (kFlagRadiiSafe)
    int32_t accum_log2 = vcrt::kAccumMaxScaleLog2;  // the scale s pixels start at (flags)
    float4* d_geom = nullptr;  // pair-SoA groups of four (+1 padding group)
    float4* d_center_radius = nullptr;
    float4* d_shade = nullptr;
    float4* d_material = nullptr;  // (material id, 1 / param, Schlick r0^2, 0) per sphere
    // culled-scan tables (cluster.hpp); ncgroups == 0 when culling does not apply
    int32_t ncgroups = 0, ncbig = 0;
    float cmargin[4] = {0, 0, 0, 0};  // box margin constants (CullTables::margin)
    float4* d_cgroup = nullptr;
    float4* d_cbound = nullptr;
    float4* d_cbound_nf = nullptr;
    float4* d_cnode = nullptr;
    float4* d_cnode_nf = nullptr;  // node-pair boxes, near/far layout, padded to whole chunks
    float4* d_ctop = nullptr;
    uint32_t* d_prim_info = nullptr;  // camera-ray tile lists (primary.cpp), flat scan only
    uint16_t* d_prim_ids = nullptr;
    float4* d_cam_rec = nullptr;  // camera-relative records: big groups, sphere lists
    bool primary_lists = true;        // VCRT_PRIMARY_LISTS=0 turns them off
    // work decomposition
    int32_t quantum = 1;  // the accumulation quantum G (a power of two)
    int32_t chunk = 1, nchunks = 1;
    int32_t tail_start = 0, tail_chunk = 1, tail_nchunks = 0;  // TraceParams' tail
    uint32_t total_pixels = 0, total_items = 0;
    bool direct = false;  // one item per pixel, not progressive: lanes write pixels (kFlagDirect)
    double* d_accum = nullptr;  // [total_pixels][4] exact sums of the quantized chunk sums
    // d_accum holds zeros: a memset, or the last resolve wrote them back (vcrt_resolve
    // zero_accum), so a non-progressive frame needs no memset of its own
    bool accum_clean = false;
    // Outlier quanta (vcrt_math.h "Accumulation"): [total_pixels] the float bits of each pixel's
    // largest |quantum sum| that passed 2^12 (0: none); once one has, every frame of the
    // configuration quantizes each pixel at its own scale (pixel_scale, kFlagPixelScale)
    uint32_t* d_pixel_emax = nullptr;
    bool pixel_scale = false;
    int32_t min_scale = vcrt::kAccumMaxScaleLog2;  // the smallest pixel scale so far
    uint64_t accumulated = 0;               // samples per pixel accumulated (progressive)
    // the host's jitter (jx, jy) of a frame's sample indices: two pinned buffers used in turn,
    // each reused only once the copy recorded by its event is done (progressive frames set up
    // their jitter without waiting for the stream)
    float2* h_jitter[2] = {nullptr, nullptr};
    hipEvent_t ev_jitter[2] = {nullptr, nullptr};
    int jitter_slot = 0;
    float* d_srgb_thresholds = nullptr;
    uchar4* d_srgb = nullptr;
    // per-frame inputs / outputs
    float2* d_jitter_in = nullptr;  // the host's jitter (jx, jy) of the frame's sample indices
    float4* d_jitter = nullptr;     // TraceParams.jitter (vcrt_setup_jitter)
    float4* d_corner = nullptr;     // TraceParams.corner (vcrt_setup_jitter, at vcrt_begin)
    float4* d_fb_own = nullptr;
    float4* d_fb = nullptr;  // current render target (own or caller-provided)
    size_t fb_bytes = 0;
    void* d_counters = nullptr;
    // the counters' first four u64 (outlier max, segments, work tallies), read back each frame:
    // host-pinned, written by vcrt_resolve (which then zeroes d_counters: counters_clean) or
    // copied when no resolve runs
    unsigned long long* h_counters = nullptr;
    bool counters_clean = false;
    uint32_t tiles_x = 0, local_tiles = 0;
    uint32_t local_elems = 0;   // float4 elements of the rank-local framebuffer
    uint64_t local_pixels = 0;  // frame pixels this rank renders
    uint32_t pad_tiles = 0;     // tiles of the largest rank: the packed framebuffers' size
    // multi-GPU, one process per GPU (vcrt_comm_init): the ranks' packed framebuffers go to
    // rank 0 in one grouped RCCL send/recv inside vcrt_draw_next_frame; rank 0 assembles them
    ncclComm_t comm = nullptr;  // non-blocking (comm_wait.hpp): every wait has a deadline
    bool comm_lost = false;     // the communicator failed or timed out and was aborted: every
                                // later draw returns VK_ERROR_DEVICE_LOST (until vcrt_begin)
    float4* d_gather = nullptr;  // rank 0: [world][pad_tiles][64], its own tiles in slot 0
    float4* d_frame = nullptr;   // rank 0: the assembled frame [height][width]
    hipEvent_t ev_gather_start = nullptr, ev_gather = nullptr;
    vcrt::Camera cam{};
    vcrt_stats stats{};
};

RendererState g;

#define VCRT_TRY(expr)                          \
    do {                                        \
        hipError_t e_ = (expr);                 \
        if (e_ != hipSuccess) return to_vk(e_); \
    } while (0)

// Samples per work item when the caller leaves it to us: 64, halved (down to 16) while the
// largest rank's share of the frame would be fewer than kChunkItems = 2^24 - 2^21 items (~45 per
// lane of the persistent grid, ~330k lanes on MI355X); at least spp / 512 (at most
// kAccumMaxChunks chunks per pixel). Smaller items cost more than they save in balance: every
// item start and end (slot fetch, pixel set-up, three f64 atomics whose completion later loads
// wait for) is paid by the whole wave, and the tail of the partition (work_tail) now absorbs the
// drain that small items used to shorten. Measured at round 2 with the tail
// (profiles/r02_tail_sweep.txt, kernel ms per rank at the C4 workload): one GPU K = 64 127.0 /
// K = 32 129.3 -> 64; 2-way shards 64.3 / 65.2 -> 64; 4-way K = 32 33.4 / K = 16 33.9 -> 32;
// 8-way K = 16 17.6 / K = 32 17.7-18.1 -> 16; C3 (256 spp) K = 32 33.55 / K = 16 33.80 -> 32.
// All ranks of a frame use the same K (the largest rank's share decides); the image depends on
// the accumulation quantum alone (work_quantum), whatever K and the tail are.
// Round 3 stopped small frames (fewer than 2^22 items at K = 32) at K = 32, measured then at C2
// (K = 32 1.35 ms against K = 16 1.47 ms, when the item was also the accumulation quantum and
// every item end read its ring entry back). Round 4 dropped that floor: with the quantum
// decoupled and the claim-time ring clearing, C2 takes 0.878-0.894 ms at K = 16 against
// 0.936-0.959 at K = 32 (K = 8: 0.882-0.896; profiles/r04_ab_log.md).
constexpr uint64_t kChunkItems = (uint64_t{1} << 24) - (uint64_t{1} << 21);
// Round 5: also halved (down to 16) while a pixel has fewer than kMinChunksPerPixel items: a
// block (64 items, all chunks of 64 / nchunks pixels) then spans few pixels, so the wave's
// 14-entry accumulation ring covers the pixels of its last ~3 blocks and long items keep their
// entries (C3: K = 32 gave 9-pixel blocks, and most quanta missed the ring: 2.5 GB of atomics
// per frame; VCRT_CHUNK_RULE=items restores the item-count rule alone).
constexpr int32_t kMinChunksPerPixel = 16;
// Round 5, the cost partition: where the item count would halve K below the per-pixel rule's K
// (the 8- and 4-way shards of C4), K stays at the per-pixel rule's value, the partition has no
// tail and the frame runs the cost order (vcrt_draw_next_frame): the last items of a sharded frame
// are then cheap ones, not the deep pixels whose 64-sample items outlast the queue by ~3 ms
// (profiles/r05_ab_log.md: 8-way max rank 11.78 ms against 12.16 with K = 16 + 128 x 4, 4-way
// 22.94 against 23.11). `allow_cost`: the desc may take it (cost_allowed); `cost` (may be null)
// reports whether it does.
int32_t default_chunk(uint64_t rank_slots, int32_t spp, bool allow_cost = false,
                      bool* cost = nullptr) {
    const char* rule = std::getenv("VCRT_CHUNK_RULE");
    const bool per_pixel = !(rule && std::strcmp(rule, "items") == 0);
    int32_t k = kDefaultChunk;
    // the per-pixel rule, then the item-count rule (both conditions are monotone in K)
    while (k > 16 && per_pixel && spp / k < kMinChunksPerPixel) k /= 2;
    const int32_t k_pixel = k;
    while (k > 16 && rank_slots * static_cast<uint64_t>((spp + k - 1) / k) < kChunkItems) k /= 2;
    const bool c = allow_cost && k < k_pixel;
    if (cost) *cost = c;
    if (c) k = k_pixel;
    const int32_t k_min = (spp + vcrt::kAccumMaxChunks - 1) / vcrt::kAccumMaxChunks;
    return std::max(k, k_min);
}

// 8x8 tiles of a W x H frame owned by `rank`: (tx, ty) with (tx + ty) % world == rank
// (vcrt_math.h tile_of / owner_of).
uint32_t tiles_for_rank(int32_t width, int32_t height, int32_t world, int32_t rank) {
    const uint32_t tiles_x = static_cast<uint32_t>((width + 7) / 8);
    const uint32_t tiles_y = static_cast<uint32_t>((height + 7) / 8);
    uint64_t n = 0;
    for (uint32_t ty = 0; ty < tiles_y; ty++)
        n += vcrt::tiles_in_row((static_cast<uint32_t>(rank) + static_cast<uint32_t>(world) -
                                 ty % static_cast<uint32_t>(world)) %
                                    static_cast<uint32_t>(world),
                                tiles_x, static_cast<uint32_t>(world));
    return static_cast<uint32_t>(n);
}

// The accumulation quantum G (vcrt.h accumulate_quantum): the image depends on G alone. A
// pixel's samples are summed in fp32 within each run of G consecutive samples, and the runs'
// sums are quantized and added exactly (vcrt_math.h "Accumulation"), at most kAccumMaxChunks of
// them per pixel: 4, doubled while the frame's samples would need more. G does not depend on
// the number of GPUs, so a sharded frame equals the one-GPU frame bit for bit with default descs
// (round 4; before, the chunk was the quantum and followed the rank's share: K = 64 on one GPU,
// 16 at N = 8, so the default images differed). Work items (chunks, the tail) hold whole quanta,
// so G bounds the tail's item size from below, which sets the drain at N = 8: with G = 4 the
// default partitions are round 3's (K = 64 + 64 x 8 on one GPU, K = 16 + 128 x 4 at N = 8);
// measured at C4, the 8-way max rank 13.42 / 13.48 / 14.39 ms with G = 4 / 8 / 16, and the one-GPU
// frame within 0.5% for the three (profiles/r04_ab_log.md).
constexpr int32_t kDefaultQuantum = 4;

int32_t work_quantum(const vcrt_render_desc& d) {
    if (d.accumulate_quantum > 0) return d.accumulate_quantum;
    int32_t q = kDefaultQuantum;
    while ((d.samples_per_pixel + q - 1) / q > vcrt::kAccumMaxChunks) q *= 2;
    return q;
}

int32_t round_up(int32_t x, int32_t q) { return static_cast<int32_t>((int64_t{x} + q - 1) / q * q); }

uint32_t max_rank_tiles(const vcrt_render_desc& d) {
    uint32_t max_tiles = 0;
    for (int32_t rr = 0; rr < d.world_size; rr++)
        max_tiles = std::max(max_tiles, tiles_for_rank(d.width, d.height, d.world_size, rr));
    return max_tiles;
}

// Whether a desc may take the cost partition (default_chunk): chunk and tail left to the rules, a
// kernel variant with a cost-order build (the linear and flat scans; AUTO picks one of them), and
// no static order asked for (VCRT_WORK_ORDER set to anything but "cost").
bool cost_allowed(const vcrt_render_desc& d) {
    if (d.accumulate_chunk > 0 || d.accumulate_tail != 0) return false;
    if (d.kernel_variant != VCRT_KERNEL_AUTO && d.kernel_variant != VCRT_KERNEL_SMEM &&
        d.kernel_variant != VCRT_KERNEL_LDS && d.kernel_variant != VCRT_KERNEL_CULL_FLAT)
        return false;
    const char* order = std::getenv("VCRT_WORK_ORDER");
    return !order || std::strcmp(order, "cost") == 0;
}

bool cost_partition(const vcrt_render_desc& d) {
    bool cost = false;
    (void)default_chunk(64ull * max_rank_tiles(d), d.samples_per_pixel, cost_allowed(d), &cost);
    return cost;
}

// Samples per work item for a desc: its accumulate_chunk, else the default for the largest rank's
// share of the frame; rounded up to whole quanta and capped at spp.
int32_t work_chunk(const vcrt_render_desc& d) {
    const int32_t k = d.accumulate_chunk > 0
                          ? d.accumulate_chunk
                          : default_chunk(64ull * max_rank_tiles(d), d.samples_per_pixel,
                                          cost_allowed(d));
    return std::min(round_up(k, work_quantum(d)), d.samples_per_pixel);
}

// The tail of the partition (vcrt.h vcrt_work_tail): the last T samples of every pixel in items
// of KT samples, handed out after the head. An item started just before the queue drains runs to
// its end while the rest of the chip idles, and its latency is K samples' worth of wave
// iterations (~13 us each at full occupancy: up to ~2 ms at K = 16, ~8 ms at K = 64). The tail
// keeps every lane busy with short items until the head's last items are done, so the head must
// cover ~6 of its items per lane: T ~ 6 K L / P for the L = 327680 lanes of the persistent grid and
// the P pixel slots of the largest rank. Measured at C4 (profiles/r02_tail_sweep.txt, kernel ms):
// one GPU K = 64 128.2 -> 127.0 with T = 64, KT = 8; 8-way shards K = 16 18.0 -> 17.6 with
// T = 128, KT = 4 (a head of K = 64 stays above 21 ms at N = 8 with any tail up to 384).
constexpr uint64_t kTailLaneItems = 6ull * 327680ull;

int32_t work_tail(const vcrt_render_desc& d, int32_t chunk, int32_t* tail_chunk) {
    const int32_t spp = d.samples_per_pixel;
    const int32_t q = work_quantum(d);
    *tail_chunk = 1;
    if (d.accumulate_tail < 0 || chunk >= spp) return 0;
    int32_t t = 0, kt = d.accumulate_tail_chunk;
    if (d.accumulate_tail > 0) {
        t = std::min(d.accumulate_tail, spp - 1);
    } else {
        if (cost_partition(d)) return 0;  // the cost order runs the cheap items last instead
        const uint32_t max_tiles = max_rank_tiles(d);
        // none when the head alone gives every lane many items (>= 2 kChunkItems: ~90 per lane):
        // the drain is then a small part of the frame and the tail's short items cost more than
        // they save. Measured round 5 (tools/ab.py, kernel ms, same bits): one GPU C4 89.68 ->
        // 89.40 without the tail, C3 23.52 -> 23.14, C5 2518 -> 2497; with it, C4 2-way shards
        // 45.18 against 46.07 and 4-way 23.21 against 23.33, 8-way 12.01 against 12.16.
        const uint64_t head_items = 64ull * max_tiles *
                                    static_cast<uint64_t>((spp + chunk - 1) / chunk);
        if (head_items >= 2ull * kChunkItems) return 0;
        const double raw = static_cast<double>(kTailLaneItems) * chunk / (64.0 * max_tiles);
        if (raw < 1.0) return 0;
        t = 1 << static_cast<int>(std::lround(std::log2(raw)));  // nearest power of two
        if (4 * static_cast<int64_t>(t) > spp) return 0;
    }
    // whole quanta: the head ends on a quantum boundary (the tail grows to it), tail items of
    // max(4, K / 8) samples (the rule) or as given, rounded up to whole quanta, the last one
    // ending at spp
    const int32_t head_end = (spp - t) / q * q;
    if (head_end <= 0) return 0;
    t = spp - head_end;
    kt = round_up(kt <= 0 ? std::max(4, chunk / 8) : kt, q);
    *tail_chunk = std::min(kt, t);
    return t;
}

// A multiplier m with (i * m) >> 32 == i / n for every item index i < 64 n of a part (the
// chunk-minor slot split, TraceParams.nch_magic), checked here for every such i; 0 when there is
// none (n <= 1, or n too large for the error term).
uint32_t division_magic(uint32_t n) {
    if (n <= 1u || n > 8192u) return 0u;
    const uint64_t m = ((uint64_t{1} << 32) + n - 1u) / n;  // ceil(2^32 / n) < 2^32
    for (uint64_t i = 0; i < 64ull * n; i++)
        if (((i * m) >> 32) != i / n) return 0u;
    return static_cast<uint32_t>(m);
}

// Jitter of sample indices base .. base+n-1 (shader.comp:48 depends only on the index).
void make_jitter(uint64_t base, int n, float2* out) {
    for (int k = 0; k < n; k++) {
        const float i = static_cast<float>(base + k), i1 = static_cast<float>(base + k + 1);
        out[k].x = vcrt::kJitterOffset + vcrt::rand2(i, i);  // shader.comp:48
        out[k].y = vcrt::kJitterOffset + vcrt::rand2(i1, i1);
    }
}

// sRGB8 thresholds: T_k = the smallest float >= the linear value whose exact sRGB encode is
// (k - 0.5) / 255, k = 1..255, so that #{k : c >= T_k} is round-to-nearest of 255 * encode(c).
void srgb_thresholds(float out[255]) {
    for (int k = 1; k <= 255; k++) {
        const double s = (k - 0.5) / 255.0;
        const double lin = s <= 0.04045 ? s / 12.92 : std::pow((s + 0.055) / 1.055, 2.4);
        float t = static_cast<float>(lin);
        if (static_cast<double>(t) < lin) t = std::nextafter(t, 2.0f);
        out[k - 1] = t;
    }
}

// Directory of this shared object (for the default code-object path).
std::string library_dir() {
    Dl_info info;
    if (dladdr(reinterpret_cast<void*>(&tiles_for_rank), &info) && info.dli_fname) {
        std::string p(info.dli_fname);
        const size_t slash = p.find_last_of('/');
        if (slash != std::string::npos) return p.substr(0, slash);
    }
    return ".";
}

// pixel00, delta_u, delta_v, centre: TraceParams.cam
std::array<float, 12> camera_array() {
    const vcrt::f3 v[4] = {g.cam.pixel00, g.cam.delta_u, g.cam.delta_v, g.cam.center};
    std::array<float, 12> c{};
    for (int i = 0; i < 4; i++) {
        c[3 * i + 0] = v[i].x;
        c[3 * i + 1] = v[i].y;
        c[3 * i + 2] = v[i].z;
    }
    return c;
}

void free_scene() {
    if (g.d_geom) (void)hipFree(g.d_geom);
    if (g.d_center_radius) (void)hipFree(g.d_center_radius);
    if (g.d_shade) (void)hipFree(g.d_shade);
    if (g.d_material) (void)hipFree(g.d_material);
    g.d_geom = nullptr;
    g.d_center_radius = nullptr;
    g.d_shade = nullptr;
    g.d_material = nullptr;
    if (g.d_cgroup) (void)hipFree(g.d_cgroup);
    if (g.d_cbound) (void)hipFree(g.d_cbound);
    if (g.d_cbound_nf) (void)hipFree(g.d_cbound_nf);
    if (g.d_cnode) (void)hipFree(g.d_cnode);
    if (g.d_cnode_nf) (void)hipFree(g.d_cnode_nf);
    if (g.d_ctop) (void)hipFree(g.d_ctop);
    if (g.d_prim_info) (void)hipFree(g.d_prim_info);
    if (g.d_prim_ids) (void)hipFree(g.d_prim_ids);
    if (g.d_cam_rec) (void)hipFree(g.d_cam_rec);
    g.d_cam_rec = nullptr;
    g.d_prim_info = nullptr;
    g.d_prim_ids = nullptr;
    g.d_cgroup = nullptr;
    g.d_cbound = nullptr;
    g.d_cbound_nf = nullptr;
    g.d_cnode = nullptr;
    g.d_cnode_nf = nullptr;
    g.d_ctop = nullptr;
    g.ncgroups = 0;
    g.ncbig = 0;
    g.nspheres = 0;
}

// A pair-SoA box table (cluster.hpp: 16 floats per pair of boxes) in the near/far layout of
// TraceParams.cbound_nf (20 floats per pair: per axis lo0 lo1 hi0 hi1 lo0 lo1, then K0 K1),
// uploaded to a new device buffer.
hipError_t upload_near_far(const std::vector<float>& pairs, float4** out) {
    const size_t n = pairs.size() / 16;
    std::vector<float> nf(n * 20);
    for (size_t i = 0; i < n; i++) {
        const float* b = &pairs[i * 16];
        float* o = &nf[i * 20];
        for (int a = 0; a < 3; a++) {  // lo of axis a at b[2a], hi at b[6 + 2a]
            o[6 * a + 0] = o[6 * a + 4] = b[2 * a];
            o[6 * a + 1] = o[6 * a + 5] = b[2 * a + 1];
            o[6 * a + 2] = b[6 + 2 * a];
            o[6 * a + 3] = b[6 + 2 * a + 1];
        }
        o[18] = b[12];
        o[19] = b[13];
    }
    hipError_t e = hipMalloc(out, sizeof(float) * nf.size());
    if (e != hipSuccess) return e;
    return hipMemcpy(*out, nf.data(), sizeof(float) * nf.size(), hipMemcpyHostToDevice);
}

// hipModuleGetFunction of a required entry point: a code object without it (e.g. an A/B build of
// an older tree) is an incompatible shader binary, not an unknown error (hipErrorNotFound used to
// map to VK_ERROR_UNKNOWN: profiles/r04_ab_log.md, run 7)
#define VCRT_BIND(fn, m, name)                                                   \
    do {                                                                         \
        const hipError_t e_ = hipModuleGetFunction(fn, m, name);                 \
        if (e_ == hipErrorNotFound) return VK_ERROR_INCOMPATIBLE_SHADER_BINARY_EXT; \
        if (e_ != hipSuccess) return to_vk(e_);                                  \
    } while (0)

VkResult bind_kernels() {
    hipModule_t m = static_cast<hipModule_t>(g.stage.module);
    VCRT_BIND(&g.k_trace_lds, m, "vcrt_trace_lds");
    VCRT_BIND(&g.k_trace_smem, m, "vcrt_trace_smem");
    VCRT_BIND(&g.k_assemble, m, "vcrt_assemble");
    VCRT_BIND(&g.k_fill, m, "vcrt_fill");
    VCRT_BIND(&g.k_resolve, m, "vcrt_resolve");
    VCRT_BIND(&g.k_encode, m, "vcrt_encode_srgb8");
    VCRT_BIND(&g.k_setup_jitter, m, "vcrt_setup_jitter");
    VCRT_BIND(&g.k_trace_lds_stats, m, "vcrt_trace_lds_stats");
    VCRT_BIND(&g.k_trace_smem_stats, m, "vcrt_trace_smem_stats");
    VCRT_BIND(&g.k_trace_cull, m, "vcrt_trace_cull");
    VCRT_BIND(&g.k_trace_cull_stats, m, "vcrt_trace_cull_stats");
    VCRT_BIND(&g.k_trace_cull_lane_lds, m, "vcrt_trace_cull_lane_lds");
    VCRT_BIND(&g.k_trace_cull_lane_lds_stats, m, "vcrt_trace_cull_lane_lds_stats");
    VCRT_BIND(&g.k_trace_cull_lane, m, "vcrt_trace_cull_lane");
    VCRT_BIND(&g.k_trace_cull_lane_stats, m, "vcrt_trace_cull_lane_stats");
    VCRT_BIND(&g.k_trace_cull_flat, m, "vcrt_trace_cull_flat");
    VCRT_BIND(&g.k_trace_cull_flat_stats, m, "vcrt_trace_cull_flat_stats");
    VCRT_BIND(&g.k_trace_cull_flat_global, m, "vcrt_trace_cull_flat_global");
    VCRT_BIND(&g.k_trace_cull_flat_global_stats, m, "vcrt_trace_cull_flat_global_stats");
    // optional: code objects built before the boxes-in-LDS flat scan lack it (A/B builds)
    if (hipModuleGetFunction(&g.k_trace_cull_flat_boxes, m, "vcrt_trace_cull_flat_boxes") !=
            hipSuccess ||
        hipModuleGetFunction(&g.k_trace_cull_flat_boxes_stats, m,
                             "vcrt_trace_cull_flat_boxes_stats") != hipSuccess) {
        (void)hipGetLastError();
        g.k_trace_cull_flat_boxes = g.k_trace_cull_flat_boxes_stats = nullptr;
    }
    // optional as well (A/B builds of earlier trees): the flat scans' cost-order builds
    const std::pair<hipFunction_t*, const char*> cost_kernels[] = {
        {&g.k_trace_cull_flat_cost, "vcrt_trace_cull_flat_cost"},
        {&g.k_trace_cull_flat_global_cost, "vcrt_trace_cull_flat_global_cost"},
        {&g.k_trace_cull_flat_boxes_cost, "vcrt_trace_cull_flat_boxes_cost"}};
    for (const auto& [fp, name] : cost_kernels)
        if (hipModuleGetFunction(fp, m, name) != hipSuccess) {
            (void)hipGetLastError();
            *fp = nullptr;
        }
    VCRT_TRY(hipModuleGetFunction(&g.k_trace_cull_lane_lds_wide, m,
                                  "vcrt_trace_cull_lane_lds_wide"));
    VCRT_TRY(hipModuleGetFunction(&g.k_trace_cull_lane_lds_wide_stats, m,
                                  "vcrt_trace_cull_lane_lds_wide_stats"));
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
    if (d.width > 65535 || d.height > 65535) return false;  // kernels pack y << 16 | x
    if (d.world_size <= 0 || d.rank < 0 || d.rank >= d.world_size) return false;
    if (d.blocks_per_cu < 0 || d.accumulate_chunk < 0) return false;
    if (d.accumulate_quantum < 0 || (d.accumulate_quantum & (d.accumulate_quantum - 1)) != 0)
        return false;  // a power of two (the kernel masks the sample index with G - 1)
    if (d.accumulate_tail < -1 || d.accumulate_tail_chunk < 0) return false;
    if (d.progressive != 0 && d.progressive != 1) return false;
    if (d.kernel_variant < VCRT_KERNEL_AUTO || d.kernel_variant > VCRT_KERNEL_CULL_FLAT) return false;
    return true;
}

// The framebuffer the caller sees: rank 0 of a gathering communicator holds the assembled
// frame [height][width]; otherwise the rank-local framebuffer.
struct FbView {
    float4* ptr;
    uint32_t elems;
};
FbView fb_view() {
    if (g.d_frame)
        return {g.d_frame, static_cast<uint32_t>(g.desc.width) * static_cast<uint32_t>(g.desc.height)};
    return {g.d_fb, g.local_elems};
}

VkResult nccl_vk(ncclResult_t e) {
    if (e == ncclSuccess) return VK_SUCCESS;
    if (e == ncclSystemError || e == ncclRemoteError) return VK_ERROR_DEVICE_LOST;
    return e == ncclInvalidArgument || e == ncclInvalidUsage ? VK_ERROR_INITIALIZATION_FAILED
                                                             : VK_ERROR_UNKNOWN;
}

template <typename Params>
VkResult launch(hipFunction_t f, uint32_t grid, uint32_t block, uint32_t lds, Params& params) {
    void* args[] = {&params};
    VCRT_TRY(hipModuleLaunchKernel(f, grid, 1, 1, block, 1, 1, lds, g.stream, args, nullptr));
    return VK_SUCCESS;
}

// Zero the pixels' sums and their outlier record (a new scene, vcrt_begin, a reset): every
// pixel starts again at the scale 2^32 (vcrt_math.h "Accumulation"). On the render stream, and
// waited for: the render stream is non-blocking, so a memset on the null stream would not be
// ordered before the next frame's kernels (a 2-GiB memset still running then zeroed the last
// rows' sums of an 8192 x 8192 frame).
hipError_t reset_sums() {
    if (g.d_accum) {
        const hipError_t e = hipMemsetAsync(g.d_accum, 0, 32u * static_cast<size_t>(g.total_pixels),
                                            g.stream);
        if (e != hipSuccess) return e;
        g.accum_clean = true;
    }
    if (g.d_pixel_emax) {
        const hipError_t e = hipMemsetAsync(
            g.d_pixel_emax, 0, sizeof(uint32_t) * static_cast<size_t>(g.total_pixels), g.stream);
        if (e != hipSuccess) return e;
    }
    if (g.stream) {
        const hipError_t e = hipStreamSynchronize(g.stream);
        if (e != hipSuccess) return e;
    }
    g.pixel_scale = false;
    g.min_scale = vcrt::kAccumMaxScaleLog2;
    g.stats.accumulate_scale_log2 = vcrt::kAccumMaxScaleLog2;
    return hipSuccess;
}

// TraceParams.jitter (vcrt_kernel_abi.h SetupJitterParams): the jitter term of the frame's
// sample indices base .. base + spp - 1 (shader.comp:48), on the device with the tracer's own
// operations.
VkResult setup_jitter(uint64_t base, bool corners = false) {
    const int spp = g.desc.samples_per_pixel;
    const int slot = g.jitter_slot;
    g.jitter_slot ^= 1;
    VCRT_TRY(hipEventSynchronize(g.ev_jitter[slot]));  // its last copy (two frames ago) is done
    make_jitter(base, spp, g.h_jitter[slot]);
    VCRT_TRY(hipMemcpyAsync(g.d_jitter_in, g.h_jitter[slot], sizeof(float2) * spp,
                            hipMemcpyHostToDevice, g.stream));
    VCRT_TRY(hipEventRecord(g.ev_jitter[slot], g.stream));
    vcrt::SetupJitterParams sp{};
    sp.jitter_in = g.d_jitter_in;
    sp.jitter = g.d_jitter;
    sp.nsamples = static_cast<uint32_t>(spp);
    const std::array<float, 12> cam = camera_array();
    for (int i = 0; i < 12; i++) sp.cam[i] = cam[i];
    sp.corner = corners ? g.d_corner : nullptr;
    sp.slots = g.total_pixels;
    sp.tiles_x = g.tiles_x;
    sp.rank = static_cast<uint32_t>(g.desc.rank);
    sp.world = static_cast<uint32_t>(g.desc.world_size);
    const uint64_t total = static_cast<uint64_t>(spp) + (sp.corner ? sp.slots : 0u);
    const uint32_t grid = static_cast<uint32_t>(std::min<uint64_t>((total + 255) / 256, 8192));
    return launch(g.k_setup_jitter, grid, 256, 0, sp);
}

// State of the non-blocking communicator's last operations (comm_wait.hpp): done, still in
// progress, or failed (an asynchronous error: a peer died, a network error).
vcrt::PollState comm_state(ncclComm_t comm) {
    ncclResult_t a = ncclSuccess;
    if (ncclCommGetAsyncError(comm, &a) != ncclSuccess) return vcrt::PollState::kFailed;
    return a == ncclSuccess      ? vcrt::PollState::kDone
           : a == ncclInProgress ? vcrt::PollState::kPending
                                 : vcrt::PollState::kFailed;
}

// Drops the communicator and the gather buffers. abort: ncclCommAbort, which also stops
// operations still running on the device (a receive whose peer is gone), so that the render
// stream drains; else a finalize (bounded) and destroy. Rank 0 renders into its own buffer again.
void comm_release(bool abort) {
    if (g.comm) {
        if (!abort) {
            const ncclResult_t f = ncclCommFinalize(g.comm);
            abort = (f != ncclSuccess && f != ncclInProgress) ||
                    vcrt::wait_with_deadline([] { return comm_state(g.comm); },
                                             vcrt::comm_timeout_ms()) != vcrt::WaitResult::kDone;
        }
        (void)(abort ? ncclCommAbort(g.comm) : ncclCommDestroy(g.comm));
        g.comm = nullptr;
    }
    if (g.stream) (void)hipStreamSynchronize(g.stream);
    if (g.d_gather) (void)hipFree(g.d_gather);
    if (g.d_frame) (void)hipFree(g.d_frame);
    if (g.ev_gather) (void)hipEventDestroy(g.ev_gather);
    if (g.ev_gather_start) (void)hipEventDestroy(g.ev_gather_start);
    g.d_gather = nullptr;
    g.d_frame = nullptr;
    g.ev_gather = nullptr;
    g.ev_gather_start = nullptr;
    g.d_fb = g.d_fb_own;
}

// A communicator failure inside a draw: abort it and report the device lost (the reference's
// errors bubble up as VkResult, VulkanComputeRayTracing.cpp:20-35).
VkResult comm_fail() {
    comm_release(true);
    g.comm_lost = true;
    return VK_ERROR_DEVICE_LOST;
}

// The frame gather, stream-ordered after the trace and resolve: every rank's
// packed tiles (pad_tiles x 64 float4, 4.1 MB per rank at 1080p / 8 GPUs) go to rank 0 in one
// grouped send/recv, so rank 0 receives from all peers at once over their own xGMI links
// (a ring all-gather would move the whole frame through every rank); rank 0 then
// re-interleaves the frame (vcrt_assemble). Every rank takes part, whatever its share. The
// communicator is non-blocking: the group is enqueued when its state leaves ncclInProgress
// (bounded wait), and the caller waits for ev_gather with a deadline (wait_gather).
VkResult gather_frame() {
    VCRT_TRY(hipEventRecord(g.ev_gather_start, g.stream));
    const size_t n = static_cast<size_t>(g.pad_tiles) * 64 * 4;  // floats per rank
    auto ok = [](ncclResult_t e) { return e == ncclSuccess || e == ncclInProgress; };
    bool good = ok(ncclGroupStart());
    if (good) {
        if (g.desc.rank == 0) {
            for (int32_t peer = 1; peer < g.desc.world_size && good; peer++)
                good = ok(ncclRecv(reinterpret_cast<float*>(g.d_gather) + n * peer, n,
                                   ncclFloat32, peer, g.comm, g.stream));
        } else {
            good = ok(ncclSend(g.d_fb, n, ncclFloat32, 0, g.comm, g.stream));
        }
        good = ok(ncclGroupEnd()) && good;
    }
    if (!good || vcrt::wait_with_deadline([] { return comm_state(g.comm); },
                                          vcrt::comm_timeout_ms()) != vcrt::WaitResult::kDone)
        return comm_fail();
    if (g.desc.rank == 0) {
        vcrt::AssembleParams ap{g.d_gather,    g.d_frame,         g.desc.width,
                                g.desc.height, g.desc.world_size, g.tiles_x,
                                g.pad_tiles};
        const uint64_t total = static_cast<uint64_t>(g.desc.width) * g.desc.height;
        const VkResult r = launch(
            g.k_assemble, static_cast<uint32_t>(std::min<uint64_t>((total + 255) / 256, 8192)),
            256, 0, ap);
        if (r != VK_SUCCESS) return r;
    }
    VCRT_TRY(hipEventRecord(g.ev_gather, g.stream));
    return VK_SUCCESS;
}

// Waits for the gather recorded by gather_frame, polling the communicator's asynchronous error
// beside the event: a peer that never sends makes this return VK_ERROR_DEVICE_LOST (after
// aborting the communicator) at the deadline instead of blocking forever.
VkResult wait_gather() {
    hipError_t ev = hipSuccess;
    const vcrt::WaitResult w = vcrt::wait_with_deadline(
        [&ev] {
            ev = hipEventQuery(g.ev_gather);
            if (ev == hipSuccess) return vcrt::PollState::kDone;
            if (ev != hipErrorNotReady) return vcrt::PollState::kFailed;
            return comm_state(g.comm) == vcrt::PollState::kFailed ? vcrt::PollState::kFailed
                                                                  : vcrt::PollState::kPending;
        },
        vcrt::gather_timeout_ms(vcrt::comm_timeout_ms(), g.stats.kernel_ms + g.stats.resolve_ms));
    if (w == vcrt::WaitResult::kDone) return VK_SUCCESS;
    if (w == vcrt::WaitResult::kFailed && ev != hipSuccess && ev != hipErrorNotReady) {
        const VkResult r = to_vk(ev);  // the device itself failed
        comm_fail();
        return r;
    }
    return comm_fail();
}

// The tracer kernel a draw launches for the current scene and desc: variant (AUTO resolved),
// entry point, block size and dynamic LDS.
struct KernelChoice {
    hipFunction_t f, stats;
    // the build a cost-ordered frame launches (it counts pixel segments into
    // TraceParams.pixel_cost and follows TraceParams.block_order); null: no cost order
    hipFunction_t cost;
    const char* name;
    uint32_t block, lds;
    int variant;
};

KernelChoice select_kernel() {
    // scan table: (groups + 1 padding group) x 64 B
    const uint32_t geom_lds = static_cast<uint32_t>(64 * ((g.nspheres + 3) / 4 + 1));
    // per-lane culled scan: tables in LDS. Up to 32 KB with 256-thread workgroups (5 per
    // CU, each with its copy); up to the CU's whole LDS with 1024-thread workgroups (one
    // copy for 16 waves); beyond that from global memory.
    const uint32_t tab_lds = static_cast<uint32_t>(16 * (g.ncgroups / 2 * 4 + g.ncgroups * 5));
    // flat: near/far boxes (80 B per pair, 336 B per node of 4 pairs: 16 B of bank padding),
    // 80-B group records (the uint16 member indices inside), the chunks' node boxes (near/far,
    // 336 B per chunk: the node level of a tracer.hip VCRT_LEVELS_NF build)
    const uint32_t tab_lds_flat = static_cast<uint32_t>(
        16 * (g.ncgroups / 8 * 21 + g.ncgroups * 5 + (g.ncgroups + 63) / 64 * 21));
    const bool lane_lds = tab_lds <= g.max_lds && g.cull_lane_tables != 2;
    const bool lane_wide = lane_lds && tab_lds > 32768u;
    int variant = g.desc.kernel_variant;
    // Measured on MI355X (1080p, box hierarchy): of the linear scans the scalar-cache
    // variant (sphere data in SGPRs, no LDS traffic) beats LDS staging by 15% (485
    // spheres) and 18% (4100); the culled scans beat both (same bits). AUTO: the flattened
    // scan (485 spheres: 3.3x SMEM, +14% over CULL_LANE, +28% over CULL; 4100 spheres with
    // its tables in global memory), and SMEM when the scene has no tables (< 16 spheres or
    // unbounded).
    if (variant == VCRT_KERNEL_AUTO)
        variant = g.ncgroups == 0 ? VCRT_KERNEL_SMEM : VCRT_KERNEL_CULL_FLAT;
    if (variant == VCRT_KERNEL_LDS && geom_lds > g.max_lds) variant = VCRT_KERNEL_SMEM;
    if ((variant == VCRT_KERNEL_CULL || variant == VCRT_KERNEL_CULL_LANE ||
         variant == VCRT_KERNEL_CULL_FLAT) &&
        g.ncgroups == 0)
        variant = VCRT_KERNEL_SMEM;
    // The flat scan keeps 4.25 KB of stacks per wave in LDS beside its tables when they fit
    // in 32 KB (16-bit entries), in 256-thread workgroups (five per CU, each with its copy of
    // the tables). Up to 1024 groups (16-bit entries) it keeps only the boxes in LDS, one copy
    // per 1024-thread workgroup; beyond that the tables stay in global memory and the stacks
    // take 32-bit entries (6.75 KB per wave).
    const bool flat_lds = tab_lds_flat <= 32768u && g.cull_lane_tables != 2 &&
                          g.cull_lane_tables != 3 && g.ncgroups <= vcrt::kFlatMaxGroups8;
    // Boxes only (near/far group boxes + node boxes of whole chunks) in LDS, one copy for the
    // 16 waves of a 1024-thread workgroup, beside their 16-bit stacks; the records from global.
    const uint32_t box_lds = static_cast<uint32_t>(
        16 * (g.ncgroups / 8 * 21 + (g.ncgroups + 63) / 64 * 21) + 16 * vcrt::kWaveScratchBytes);
    // Measured at C5 (stress scene, 4K, 4096 spp, depth 50): 11415 against 11186 Msamples/s
    // with every table in global memory (same bits; profiles/r03_c5_boxes_*).
    const bool flat_boxes = !flat_lds && g.k_trace_cull_flat_boxes != nullptr &&
                            g.cull_lane_tables != 2 && g.ncgroups <= vcrt::kFlatMaxGroups &&
                            box_lds <= g.max_lds;
    hipFunction_t f = g.k_trace_smem, fs = g.k_trace_smem_stats;
    const char* fname = "vcrt_trace_smem";
    uint32_t block = 256;
    uint32_t lds = 0;
    if (variant == VCRT_KERNEL_LDS) {
        f = g.k_trace_lds;
        fs = g.k_trace_lds_stats;
        fname = "vcrt_trace_lds";
        lds = geom_lds;
    } else if (variant == VCRT_KERNEL_CULL) {
        f = g.k_trace_cull;
        fs = g.k_trace_cull_stats;
        fname = "vcrt_trace_cull";
    } else if (variant == VCRT_KERNEL_CULL_FLAT && flat_lds) {
        f = g.k_trace_cull_flat;
        fs = g.k_trace_cull_flat_stats;
        fname = "vcrt_trace_cull_flat";
        // (experiments: a code object built with -DVCRT_FLAT_BLOCK=n launches n-thread groups)
        int max_threads = 0;  // only a code object built for that size takes it
        if (g.flat_block > 0 &&
            hipFuncGetAttribute(&max_threads, HIP_FUNC_ATTRIBUTE_MAX_THREADS_PER_BLOCK, f) ==
                hipSuccess &&
            max_threads >= g.flat_block)
            block = static_cast<uint32_t>(g.flat_block);
        lds = tab_lds_flat + (block / 64) * vcrt::kWaveScratchBytes8;
    } else if (variant == VCRT_KERNEL_CULL_FLAT && flat_boxes) {
        f = g.k_trace_cull_flat_boxes;
        fs = g.k_trace_cull_flat_boxes_stats;
        fname = "vcrt_trace_cull_flat_boxes";
        block = 1024;
        lds = box_lds;
    } else if (variant == VCRT_KERNEL_CULL_FLAT) {
        f = g.k_trace_cull_flat_global;
        fs = g.k_trace_cull_flat_global_stats;
        fname = "vcrt_trace_cull_flat_global";
        lds = 4 * vcrt::kWaveScratchBytesWide;
    } else if (variant == VCRT_KERNEL_CULL_LANE && lane_wide) {
        f = g.k_trace_cull_lane_lds_wide;
        fs = g.k_trace_cull_lane_lds_wide_stats;
        fname = "vcrt_trace_cull_lane_lds_wide";
        block = 1024;
        lds = tab_lds;
    } else if (variant == VCRT_KERNEL_CULL_LANE && lane_lds) {
        f = g.k_trace_cull_lane_lds;
        fs = g.k_trace_cull_lane_lds_stats;
        fname = "vcrt_trace_cull_lane_lds";
        lds = tab_lds;
    } else if (variant == VCRT_KERNEL_CULL_LANE) {
        f = g.k_trace_cull_lane;
        fs = g.k_trace_cull_lane_stats;
        fname = "vcrt_trace_cull_lane";
    }
    // the cost order (vcrt_draw_next_frame): the linear scans' product builds have it, the flat
    // scans have separate builds (the hooks cost the product kernel ~0.3% at C4)
    hipFunction_t fc = f == g.k_trace_smem || f == g.k_trace_lds        ? f
                       : f == g.k_trace_cull_flat                        ? g.k_trace_cull_flat_cost
                       : f == g.k_trace_cull_flat_global ? g.k_trace_cull_flat_global_cost
                       : f == g.k_trace_cull_flat_boxes  ? g.k_trace_cull_flat_boxes_cost
                                                         : nullptr;
    return KernelChoice{f, fs, fc, fname, block, lds, variant};
}

}  // namespace

extern "C" {

vcrt_result vcrt_default_desc(vcrt_render_desc* d) {
    if (!d) return VCRT_ERROR_INITIALIZATION_FAILED;
    std::memset(d, 0, sizeof(*d));
    d->struct_size = sizeof(vcrt_render_desc);
    d->width = vcrt::kRefImageWidth;  // globals.glsl:16-17
    d->height = vcrt::kRefImageHeight;
    d->samples_per_pixel = vcrt::kRefSamplesPerPixel;  // globals.glsl:9-13 (#if 0 -> 1)
    d->max_depth = vcrt::kRefMaxRecursion;             // globals.glsl:14
    std::memcpy(d->camera.lookfrom, vcrt::kRefLookfrom, sizeof(d->camera.lookfrom));  // :21-24
    std::memcpy(d->camera.lookat, vcrt::kRefLookat, sizeof(d->camera.lookat));
    std::memcpy(d->camera.vup, vcrt::kRefVup, sizeof(d->camera.vup));
    d->camera.vfov = vcrt::kRefVfov;
    d->device = -1;
    d->rank = 0;
    d->world_size = 1;
    d->kernel_variant = VCRT_KERNEL_AUTO;
    return VCRT_SUCCESS;
}

int32_t vcrt_work_chunk(const vcrt_render_desc* desc) {
    if (!desc || !desc_valid(*desc)) return VCRT_ERROR_INITIALIZATION_FAILED;
    return work_chunk(*desc);
}

int32_t vcrt_work_quantum(const vcrt_render_desc* desc) {
    if (!desc || !desc_valid(*desc)) return VCRT_ERROR_INITIALIZATION_FAILED;
    return work_quantum(*desc);
}

int32_t vcrt_work_tail(const vcrt_render_desc* desc, int32_t* tail_chunk) {
    if (!desc || !desc_valid(*desc) || !tail_chunk) return VCRT_ERROR_INITIALIZATION_FAILED;
    return work_tail(*desc, work_chunk(*desc), tail_chunk);
}

int32_t vcrt_pixel_scale_log2(float max_abs_quantum_sum) {
    const float e = std::fabs(max_abs_quantum_sum);
    uint32_t bits = 0;
    std::memcpy(&bits, &e, sizeof(bits));
    return vcrt::pixel_scale_log2(e >= 0x1p12f && std::isfinite(e) ? bits : 0u);
}

vcrt_result vcrt_begin(const vcrt_render_desc* desc) {
    if (!desc || !desc_valid(*desc)) return VCRT_ERROR_INITIALIZATION_FAILED;
    if (g.begun) vcrt_end();
    g = RendererState{};
    g.desc = *desc;
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
    g.lds_per_cu = static_cast<uint32_t>(prop.maxSharedMemoryPerMultiProcessor);
    if ((r = to_vk(hipStreamCreateWithFlags(&g.stream, hipStreamNonBlocking))) != VK_SUCCESS)
        return fail(r);
    if ((r = to_vk(hipEventCreate(&g.ev_start))) != VK_SUCCESS) return fail(r);
    if ((r = to_vk(hipEventCreate(&g.ev_stop))) != VK_SUCCESS) return fail(r);
    if ((r = to_vk(hipEventCreate(&g.ev_resolve))) != VK_SUCCESS) return fail(r);
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
    if ((r = to_vk(hipMalloc(&g.d_jitter_in, sizeof(float2) * spp))) != VK_SUCCESS) return fail(r);
    for (int k = 0; k < 2; k++) {
        if ((r = to_vk(hipHostMalloc(&g.h_jitter[k], sizeof(float2) * spp))) != VK_SUCCESS)
            return fail(r);
        if ((r = to_vk(hipEventCreateWithFlags(&g.ev_jitter[k], hipEventDisableTiming))) !=
            VK_SUCCESS)
            return fail(r);
    }
    if ((r = to_vk(hipMalloc(&g.d_jitter, sizeof(float4) * spp))) != VK_SUCCESS) return fail(r);
    {
        float th[255];
        srgb_thresholds(th);
        if ((r = to_vk(hipMalloc(&g.d_srgb_thresholds, sizeof(th)))) != VK_SUCCESS) return fail(r);
        if ((r = to_vk(hipMemcpy(g.d_srgb_thresholds, th, sizeof(th), hipMemcpyHostToDevice))) !=
            VK_SUCCESS)
            return fail(r);
    }

    // Frame sharding: 8x8 tiles, (tx, ty) to rank (tx + ty) % world (DESIGN.md "Multi-GPU").
    g.tiles_x = static_cast<uint32_t>((g.desc.width + 7) / 8);
    g.local_tiles = tiles_for_rank(g.desc.width, g.desc.height, g.desc.world_size, g.desc.rank);
    // a lane keeps its item's slot in the low kRingQBits bits of one register (the ring entry
    // above it): at most 2^26 slots per rank (8192 x 8192 on one GPU)
    if (static_cast<uint64_t>(g.local_tiles) * 64u > (uint64_t{1} << vcrt::kRingQBits))
        return fail(VCRT_ERROR_FORMAT_NOT_SUPPORTED);
    g.local_elems = g.desc.world_size == 1
                        ? static_cast<uint32_t>(g.desc.width) * static_cast<uint32_t>(g.desc.height)
                        : g.local_tiles * 64u;
    g.fb_bytes = static_cast<size_t>(g.local_elems) * sizeof(float4);
    for (int32_t rr = 0; rr < g.desc.world_size; rr++)
        g.pad_tiles = std::max(g.pad_tiles, tiles_for_rank(g.desc.width, g.desc.height,
                                                           g.desc.world_size, rr));
    for (uint32_t lt = 0; lt < g.local_tiles; lt++) {
        uint32_t tx, ty;
        vcrt::tile_of(lt, static_cast<uint32_t>(g.desc.rank),
                      static_cast<uint32_t>(g.desc.world_size), g.tiles_x, &tx, &ty);
        g.local_pixels += std::min<uint64_t>(8, g.desc.width - 8 * tx) *
                          std::min<uint64_t>(8, g.desc.height - 8 * ty);
    }
    // sharded: padded to the largest rank, the size every rank sends -- also a rank that owns
    // no tile (a frame of fewer tiles than ranks) sends that many zero bytes to the gather
    const size_t own = g.desc.world_size == 1 ? g.fb_bytes
                                              : static_cast<size_t>(g.pad_tiles) * 64 * 16;
    if (own) {
        if ((r = to_vk(hipMalloc(&g.d_fb_own, own))) != VK_SUCCESS) return fail(r);
        if ((r = to_vk(hipMemsetAsync(g.d_fb_own, 0, own, g.stream))) != VK_SUCCESS)
            return fail(r);
    }
    g.d_fb = g.d_fb_own;
    // Work decomposition: (local tile, chunk of K samples) items holding whole quanta; a pixel's
    // quantum sums are combined exactly (vcrt_math.h "Accumulation"), at most kAccumMaxChunks.
    g.total_pixels = g.local_tiles * 64u;  // local element slots incl. partial-tile padding
    // the camera-ray tables: the jitter terms and the local slots' pixel corners
    if (g.total_pixels &&
        (r = to_vk(hipMalloc(&g.d_corner, sizeof(float4) * g.total_pixels))) != VK_SUCCESS)
        return fail(r);
    if ((r = setup_jitter(0, g.total_pixels != 0)) != VK_SUCCESS) return fail(r);
    g.quantum = work_quantum(g.desc);
    if ((spp + g.quantum - 1) / g.quantum > vcrt::kAccumMaxChunks)
        return fail(VCRT_ERROR_FORMAT_NOT_SUPPORTED);
    g.chunk = work_chunk(g.desc);
    g.cost_partition = cost_partition(g.desc);
    {
        const int32_t t = work_tail(g.desc, g.chunk, &g.tail_chunk);
        g.tail_start = spp - t;
        g.tail_nchunks = t > 0 ? (t + g.tail_chunk - 1) / g.tail_chunk : 0;
    }
    g.nchunks = (g.tail_start + g.chunk - 1) / g.chunk;
    g.nch_magic[0] = division_magic(static_cast<uint32_t>(g.nchunks));
    g.nch_magic[1] = division_magic(static_cast<uint32_t>(g.tail_nchunks));
    if (g.nchunks >= 0x10000 || g.tail_nchunks >= 0x10000)  // the kernel's 16-bit chunk field
        return fail(VCRT_ERROR_FORMAT_NOT_SUPPORTED);
    // one quantum covers the pixel: the lane divides its fp32 sum (the reference's arithmetic)
    g.direct = g.quantum >= spp && !g.desc.progressive;
    {
        const uint64_t items = static_cast<uint64_t>(g.total_pixels) *
                               static_cast<uint64_t>(g.nchunks + g.tail_nchunks);
        if (items >= (uint64_t{1} << 31)) return fail(VCRT_ERROR_FORMAT_NOT_SUPPORTED);
        g.total_items = static_cast<uint32_t>(items);
    }
    if (!g.direct && g.total_pixels) {  // 32 B per pixel, whatever the spp
        const size_t bytes = 32u * static_cast<size_t>(g.total_pixels);
        if ((r = to_vk(hipMalloc(&g.d_accum, bytes))) != VK_SUCCESS) return fail(r);
        if ((r = to_vk(hipMemsetAsync(g.d_accum, 0, bytes, g.stream))) != VK_SUCCESS)
            return fail(r);
        g.accum_clean = true;
        const size_t eb = sizeof(uint32_t) * static_cast<size_t>(g.total_pixels);
        if ((r = to_vk(hipMalloc(&g.d_pixel_emax, eb))) != VK_SUCCESS) return fail(r);
        if ((r = to_vk(hipMemsetAsync(g.d_pixel_emax, 0, eb, g.stream))) != VK_SUCCESS)
            return fail(r);
    }
    if ((r = to_vk(hipMalloc(&g.d_counters, kCounterBytes))) != VK_SUCCESS) return fail(r);
    if ((r = to_vk(hipHostMalloc(&g.h_counters, 4 * sizeof(unsigned long long)))) != VK_SUCCESS)
        return fail(r);
    if (const char* e = std::getenv("VCRT_DEBUG_STATS")) g.debug_stats = std::atoi(e);
    if (const char* e = std::getenv("VCRT_PRIMARY_LISTS")) g.primary_lists = std::atoi(e) != 0;
    if (const char* e = std::getenv("VCRT_CULL_LANE_TABLES"))
        g.cull_lane_tables = std::strcmp(e, "lds") == 0      ? 1
                             : std::strcmp(e, "global") == 0 ? 2
                             : std::strcmp(e, "boxes") == 0  ? 3
                                                             : 0;
    // Blocks run from the last local tile to the first: the bottom of the frame (ground and
    // spheres, many bounces) first, the sky last, which shortens the drain at the end of the
    // queue (N = 8: 34.8 -> 33.8 ms per rank). VCRT_WORK_ORDER=forward restores top-down.
    g.work_flags |= vcrt::kFlagReverseOrder;
    if (const char* e = std::getenv("VCRT_WORK_ORDER"))
        if (std::strcmp(e, "forward") == 0) g.work_flags &= ~vcrt::kFlagReverseOrder;
    if (const char* e = std::getenv("VCRT_WORK_ORDER"))
        g.cost_order = std::strcmp(e, "cost") == 0 ? 1 : 0;  // any other value: static order
    // A block's 64 items are all the chunks of 64 / nchunks pixels (chunk-minor): the camera
    // rays of a wave then come from a few pixels (+2.8% at the C4 workload against one chunk of
    // a whole tile, same bits). VCRT_ITEM_ORDER=tile restores the tile-wide blocks.
    g.work_flags |= vcrt::kFlagChunkMinor;
    if (const char* e = std::getenv("VCRT_ITEM_ORDER"))
        if (std::strcmp(e, "tile") == 0) g.work_flags &= ~vcrt::kFlagChunkMinor;
    if (const char* e = std::getenv("VCRT_STAGE_TABLES")) g.stage_tables = std::atoi(e) != 0;
    if (const char* e = std::getenv("VCRT_FLAT_BLOCK")) {  // the LDS flat scan's group size
        const int v = std::atoi(e) / 64 * 64;
        g.flat_block = v <= 0 ? 0 : std::min(1024, v);
    }
    if (const char* e = std::getenv("VCRT_FETCH_MIN"))
        g.fetch_min = static_cast<uint32_t>(std::max(1, std::atoi(e)));
    if (const char* e = std::getenv("VCRT_FETCH_WAIT"))
        g.fetch_wait = static_cast<uint32_t>(std::max(0, std::atoi(e)));
    if (const char* e = std::getenv("VCRT_MAX_BLOCKS_PER_CU"))  // cap on the occupancy rule
        g.max_blocks_per_cu = std::max(1, std::atoi(e));
    if (const char* e = std::getenv("VCRT_ACCUM_RING")) {  // 0: off; n > 1: at most n entries
        // (clamped to kRingMaxEntries: a lane keeps its entry + 1 in the top bits of its pixel
        // index, so a larger ring would silently stop serving most pixels)
        g.accum_ring = std::atoi(e) != 0;
        if (std::atoi(e) > 1)
            g.ring_max = std::min<uint32_t>(static_cast<uint32_t>(std::atoi(e)),
                                            vcrt::kRingMaxEntries);
    }
    if (g.debug_stats && (r = to_vk(hipMalloc(&g.d_debug, sizeof(g.stats.debug)))) != VK_SUCCESS)
        return fail(r);

    // The reference's world[] is compiled in; default to the same final scene.
    std::vector<vcrt_sphere> world;
    vcrt::builtin_scene(VCRT_SCENE_FINAL, world);
    if ((r = vcrt_set_scene(world.data(), static_cast<int32_t>(world.size()))) != VK_SUCCESS)
        return fail(r);
    g.stats.local_tiles = static_cast<int32_t>(g.local_tiles);
    g.stats.accumulate_chunk = g.chunk;
    g.stats.accumulate_quantum = g.quantum;
    g.stats.accumulate_tail = spp - g.tail_start;
    g.stats.accumulate_tail_chunk = g.tail_nchunks > 0 ? g.tail_chunk : 0;
    return VCRT_SUCCESS;
}

vcrt_result vcrt_set_scene(const vcrt_sphere* spheres, int32_t count) {
    if (!g.begun) return VCRT_ERROR_INITIALIZATION_FAILED;
    if (count < 0 || (count > 0 && !spheres)) return VCRT_ERROR_INITIALIZATION_FAILED;
    // Scan table: groups of four spheres in pair-SoA form
    //   (cx0,cx1,cy0,cy1) (cz0,cz1,r0²,r1²) (cx2,cx3,cy2,cy3) (cz2,cz3,r2²,r3²),
    // r² = radius*radius as hit_sphere computes it (functions.glsl:18). The last group is
    // padded with far-away empty spheres and one extra group follows for the prefetch; the
    // kernel never accepts a padding index anyway.
    const int32_t ngroups = (count + 3) / 4;
    std::vector<float> table(static_cast<size_t>(ngroups + 1) * 16, 0.0f);
    for (int32_t j = 0; j < 4 * (ngroups + 1); j++) {
        float* gq = &table[static_cast<size_t>(j / 4) * 16];
        const int pair = (j % 4) / 2, e = j % 2;
        float cx = 0.f, cy = 0.f, cz = 0.f, r2 = -3.0e38f;
        if (j < count) {
            const vcrt_sphere& sp = spheres[j];
            cx = sp.center[0];
            cy = sp.center[1];
            cz = sp.center[2];
            r2 = sp.radius * sp.radius;
        }
        float* base = gq + 8 * pair;
        base[0 + e] = cx;
        base[2 + e] = cy;
        base[4 + e] = cz;
        base[6 + e] = r2;
    }
    std::vector<float4> cr(count), shade(count);
    std::vector<float4> mat(count);
    for (int32_t i = 0; i < count; i++) {
        const vcrt_sphere& sp = spheres[i];
        cr[i] = make_float4(sp.center[0], sp.center[1], sp.center[2], sp.radius);
        shade[i] = make_float4(sp.colour[0], sp.colour[1], sp.colour[2], sp.texture[1]);
        // the glass scatter's two per-sphere quotients (textures.glsl:49-50, functions.glsl:58-60),
        // fp32 and correctly rounded as the kernel would compute them
        const float ior = sp.texture[1];
        float r0 = (1.0f - ior) / (1.0f + ior);
        r0 = r0 * r0;
        mat[i] = make_float4(sp.texture[0], 1.0f / ior, r0, 0.0f);
    }
    vcrt::CullTables ct;
    vcrt::build_cull_tables(spheres, count, ct);
    (void)hipStreamSynchronize(g.stream);
    free_scene();
    if (ct.ngroups > 0) {
        // group records: the four pair-SoA float4s + the member indices (int bits)
        const int32_t nall = ct.nbig + ct.ngroups;  // big-sphere groups first
        std::vector<float> rec(static_cast<size_t>(nall) * 20);
        for (int32_t gi = 0; gi < nall; gi++) {
            std::memcpy(&rec[gi * 20], &ct.geom[gi * 16], 16 * sizeof(float));
            std::memcpy(&rec[gi * 20 + 16], &ct.index[gi * 4], 4 * sizeof(int32_t));
        }
        VCRT_TRY(hipMalloc(&g.d_cgroup, sizeof(float) * rec.size()));
        VCRT_TRY(hipMalloc(&g.d_cbound, sizeof(float) * ct.bound.size()));
        VCRT_TRY(hipMalloc(&g.d_cnode, sizeof(float) * ct.node.size()));
        VCRT_TRY(hipMalloc(&g.d_ctop, sizeof(float) * ct.top.size()));
        VCRT_TRY(hipMemcpy(g.d_ctop, ct.top.data(), sizeof(float) * ct.top.size(),
                           hipMemcpyHostToDevice));
        VCRT_TRY(hipMemcpy(g.d_cgroup, rec.data(), sizeof(float) * rec.size(),
                           hipMemcpyHostToDevice));
        VCRT_TRY(hipMemcpy(g.d_cbound, ct.bound.data(), sizeof(float) * ct.bound.size(),
                           hipMemcpyHostToDevice));
        // near/far layout of the group boxes for the flat scan (vcrt_kernel_abi.h, cbound_nf)
        VCRT_TRY(upload_near_far(ct.bound, &g.d_cbound_nf));
        {
            // the flat scan's chunk passes read a chunk's 4 node pairs: pad to whole chunks
            std::vector<float> nodes = ct.node;
            const size_t pairs = nodes.size() / 16, padded = (pairs + 3) / 4 * 4;
            nodes.resize(padded * 16, 0.0f);
            VCRT_TRY(upload_near_far(nodes, &g.d_cnode_nf));
        }
        VCRT_TRY(hipMemcpy(g.d_cnode, ct.node.data(), sizeof(float) * ct.node.size(),
                           hipMemcpyHostToDevice));
        g.ncgroups = ct.ngroups;
        g.ncbig = ct.nbig;
        std::memcpy(g.cmargin, ct.margin, sizeof(ct.margin));
        if (g.primary_lists && g.local_tiles > 0) {
            // camera rays of a tile start from its quarter's lists (primary.cpp): the groups
            // for the main scan, the spheres for the camera fast trace; info interleaved
            vcrt::PrimaryLists pl;
            vcrt::build_primary_lists(ct, camera_array().data(), g.desc.width, g.desc.height,
                                      g.desc.rank, g.desc.world_size, pl);
            vcrt::PrimarySphereLists sl;
            vcrt::build_primary_sphere_lists(ct, spheres, camera_array().data(), g.desc.width,
                                             g.desc.height, g.desc.rank, g.desc.world_size, sl);
            std::vector<uint32_t> info(2 * pl.info.size());
            for (size_t e = 0; e < pl.info.size(); e++) {
                info[2 * e] = pl.info[e];
                info[2 * e + 1] = sl.info[e];
            }
            VCRT_TRY(hipMalloc(&g.d_prim_info, sizeof(uint32_t) * info.size()));
            VCRT_TRY(hipMemcpy(g.d_prim_info, info.data(), sizeof(uint32_t) * info.size(),
                               hipMemcpyHostToDevice));
            VCRT_TRY(hipMalloc(&g.d_prim_ids, sizeof(uint16_t) * (pl.ids.size() + 1)));
            if (!pl.ids.empty())
                VCRT_TRY(hipMemcpy(g.d_prim_ids, pl.ids.data(), sizeof(uint16_t) * pl.ids.size(),
                                   hipMemcpyHostToDevice));
            // the camera fast trace's records: the big groups', then the sphere lists' pairs
            std::vector<float> crec;
            vcrt::build_camera_records(ct, camera_array().data(), crec);
            crec.resize(static_cast<size_t>(ct.nbig) * 16);
            crec.insert(crec.end(), sl.rec.begin(), sl.rec.end());
            crec.resize(crec.size() + 12, 0.0f);  // never empty
            VCRT_TRY(hipMalloc(&g.d_cam_rec, sizeof(float) * crec.size()));
            VCRT_TRY(hipMemcpy(g.d_cam_rec, crec.data(), sizeof(float) * crec.size(),
                               hipMemcpyHostToDevice));
        }
    }
    VCRT_TRY(hipMalloc(&g.d_geom, sizeof(float) * table.size()));
    VCRT_TRY(hipMemcpy(g.d_geom, table.data(), sizeof(float) * table.size(),
                       hipMemcpyHostToDevice));
    if (count > 0) {
        VCRT_TRY(hipMalloc(&g.d_center_radius, sizeof(float4) * count));
        VCRT_TRY(hipMalloc(&g.d_shade, sizeof(float4) * count));
        VCRT_TRY(hipMalloc(&g.d_material, sizeof(float4) * count));
        VCRT_TRY(hipMemcpy(g.d_center_radius, cr.data(), sizeof(float4) * count,
                           hipMemcpyHostToDevice));
        VCRT_TRY(
            hipMemcpy(g.d_shade, shade.data(), sizeof(float4) * count, hipMemcpyHostToDevice));
        VCRT_TRY(
            hipMemcpy(g.d_material, mat.data(), sizeof(float4) * count, hipMemcpyHostToDevice));
    }
    // (the uploads above ran on the null stream; the render stream does not wait for it)
    VCRT_TRY(hipStreamSynchronize(nullptr));
    g.nspheres = count;
    g.stats.nspheres = count;
    if (g.desc.progressive && g.accumulated > 0) {
        // a new scene restarts progressive accumulation at sample 0: the jitter table holds
        // the last frame's sample indices
        const VkResult rj = setup_jitter(0);
        if (rj != VK_SUCCESS) return rj;
    }
    g.accumulated = 0;
    g.order_key = 0;    // and its cost order is measured again
    VCRT_TRY(reset_sums());
    g.scene_bounded = true;
    g.radii_safe = true;
    for (int32_t i = 0; i < count; i++) {
        const vcrt_sphere& sp = spheres[i];
        for (float v : {sp.center[0], sp.center[1], sp.center[2], sp.radius})
            if (!(std::fabs(v) <= 0x1p30f)) g.scene_bounded = false;  // also rejects NaN
        if (!(std::fabs(sp.radius) >= 0x1p-40f && std::fabs(sp.radius) <= 0x1p30f))
            g.radii_safe = false;
    }
    g.stage.pName = select_kernel().name;  // the entry point draws of this scene dispatch
    return VCRT_SUCCESS;
}

// Cost order (vcrt_draw_next_frame): at most this many items per lane of the persistent grid
// make a frame drain-bound (C2: 3.7; C3, C4 on one GPU: ~100; C4 8-way shards: ~50).
constexpr uint64_t kCostOrderItemsPerLane = 8;
// Waves per SIMD of such frames (C2, measured round 5: 0.792 ms at 6 waves, 0.763-0.769 at 5,
// 0.773 at 4, with the cost order; 0.829 / 0.797 without it).
constexpr uint32_t kDrainWavesPerSimd = 5;

// The configuration a measured order belongs to: kernel, grid and partition (a new scene or
// vcrt_begin resets it through order_key = 0).
uint64_t order_key_of(hipFunction_t f, uint32_t grid, uint32_t total_blocks) {
    uint64_t h = 1469598103934665603ull;
    auto mix = [&h](uint64_t v) { h = (h ^ v) * 1099511628211ull; };
    mix(reinterpret_cast<uintptr_t>(f));
    mix(grid);
    mix(total_blocks);
    mix(static_cast<uint64_t>(g.nchunks));
    mix(static_cast<uint64_t>(g.tail_nchunks));
    mix(g.local_tiles);
    return h | 1u;
}

// From the pixels' segment counts of the frame just rendered: every block (head and tail
// together) by decreasing cost of its items, longest first (the makespan heuristic), so that the
// items still running when the queue drains are the shortest: the tail's items of cheap pixels.
// A block's item cost is the mean segment count of the pixels its 64 chunk-minor items belong to
// (item i of tile lt's part with n chunks per pixel: slot i / n) times the part's samples per
// item; ties in the static order (head, then tail, each bottom-up: the highest block first).
VkResult build_block_order(uint32_t total_blocks) {
    std::vector<uint32_t> cost(g.total_pixels);
    VCRT_TRY(hipMemcpy(cost.data(), g.d_pixel_cost, cost.size() * sizeof(uint32_t),
                       hipMemcpyDeviceToHost));
    std::vector<uint32_t> order(total_blocks);
    std::vector<uint64_t> bc(total_blocks, 0);
    const uint32_t head = g.local_tiles * static_cast<uint32_t>(g.nchunks);
    auto part = [&](uint32_t base, uint32_t nblocks, uint32_t nch, uint32_t samples) {
        for (uint32_t b = 0; b < nblocks; b++) {
            const uint32_t lt = b / nch, c = b - lt * nch;
            // chunk-minor: slots (64 c) / nch .. (64 c + 63) / nch; tile-wide blocks
            // (VCRT_ITEM_ORDER=tile): one chunk of all 64 slots
            const bool cm = (g.work_flags & vcrt::kFlagChunkMinor) != 0u;
            const uint32_t s0 = cm ? (64u * c) / nch : 0u;
            const uint32_t s1 = cm ? std::min((64u * c + 63u) / nch, 63u) : 63u;
            uint64_t sum = 0;
            for (uint32_t sl = s0; sl <= s1; sl++) sum += cost[lt * 64u + sl];
            bc[base + b] = sum * samples * 64u / (s1 - s0 + 1u);
        }
    };
    if (head > 0)
        part(0, head, static_cast<uint32_t>(g.nchunks), static_cast<uint32_t>(g.chunk));
    if (total_blocks > head)
        part(head, total_blocks - head, static_cast<uint32_t>(g.tail_nchunks),
             static_cast<uint32_t>(g.tail_chunk));
    uint32_t k = 0;
    for (uint32_t b = head; b-- > 0;) order[k++] = b;
    for (uint32_t b = total_blocks; b-- > head;) order[k++] = b;
    std::stable_sort(order.begin(), order.end(),
                     [&bc](uint32_t x, uint32_t y) { return bc[x] > bc[y]; });
    if (total_blocks > g.order_words) {
        if (g.d_block_order) (void)hipFree(g.d_block_order);
        g.d_block_order = nullptr;
        g.order_words = 0;
        VCRT_TRY(hipMalloc(&g.d_block_order, total_blocks * sizeof(uint32_t)));
        g.order_words = total_blocks;
    }
    VCRT_TRY(hipMemcpy(g.d_block_order, order.data(), total_blocks * sizeof(uint32_t),
                       hipMemcpyHostToDevice));
    VCRT_TRY(hipStreamSynchronize(nullptr));  // before the render stream's next frame reads it
    return VK_SUCCESS;
}

// One render of the frame's samples (the tracer kernel and, when the pixels sum quanta, the
// resolve pass) on the render stream, waited for; *outlier_max receives the float bits of the
// largest |quantum sum| that did not fit its pixel's scale (0: none; vcrt_math.h
// "Accumulation").
static VkResult trace_frame(uint64_t spp_total, uint32_t* outlier_max) {
    const uint32_t pixels = g.total_pixels;
    vcrt::TraceParams p{};
    p.geom = g.d_geom;
    p.center_radius = g.d_center_radius;
    p.shade = g.d_shade;
    p.material = g.d_material;
    p.jitter = g.d_jitter;
    p.corner = g.d_corner;
    p.out = g.d_fb;
    p.accum = g.d_accum;
    p.work = reinterpret_cast<uint32_t*>(static_cast<char*>(g.d_counters) + 256);
    p.segments = reinterpret_cast<unsigned long long*>(static_cast<char*>(g.d_counters) + 8);
    p.debug = static_cast<unsigned long long*>(g.d_debug);
    p.work_done = reinterpret_cast<unsigned long long*>(static_cast<char*>(g.d_counters) + 16);
    p.cgroup = g.d_cgroup;
    p.cbound = g.d_cbound;
    p.cbound_nf = g.d_cbound_nf;
    p.cnode = g.d_cnode;
    p.cnode_nf = g.d_cnode_nf;
    p.ctop = g.d_ctop;
    p.prim_info = g.d_prim_info;
    p.prim_ids = g.d_prim_ids;
    p.cam_rec = g.d_cam_rec;
    p.ncgroups = g.ncgroups;
    p.nbig = g.ncbig;
    for (int k = 0; k < 4; k++) p.box_margin[k] = g.cmargin[k];
    p.nspheres = g.nspheres;
    p.width = g.desc.width;
    p.height = g.desc.height;
    p.spp = g.desc.samples_per_pixel;
    p.max_depth = g.desc.max_depth;
    p.rank = g.desc.rank;
    p.world = g.desc.world_size;
    p.tiles_x = g.tiles_x;
    p.local_tiles = g.local_tiles;
    p.total_items = g.total_items;
    p.chunk = g.chunk;
    p.quantum_mask = static_cast<uint32_t>(g.quantum - 1);
    p.nchunks = g.nchunks;
    p.tail_start = g.tail_start;
    p.tail_chunk = g.tail_chunk;
    p.tail_nchunks = g.tail_nchunks;
    p.blocks_head = g.local_tiles * static_cast<uint32_t>(g.nchunks);
    p.flags = g.work_flags | (g.scene_bounded ? vcrt::kFlagSceneBounded : 0u) |
              (g.radii_safe ? vcrt::kFlagRadiiSafe : 0u) |
              (g.direct ? vcrt::kFlagDirect : 0u) |
              (g.pixel_scale ? vcrt::kFlagPixelScale : 0u) |
              (static_cast<uint32_t>(g.accum_log2 + vcrt::kFlagScaleBias)
               << vcrt::kFlagScaleShift);
    // outlier quanta (vcrt_math.h "Accumulation"); the kernel's quantizing retire writes them
    p.pixel_emax = g.d_pixel_emax;
    p.outlier_max = static_cast<uint32_t*>(g.d_counters);  // u32 at 0 (zeroed every launch)
    if (!g.direct && (p.pixel_emax == nullptr || g.d_accum == nullptr))
        return VK_ERROR_INITIALIZATION_FAILED;
    p.spp_total = static_cast<float>(spp_total);
    p.region = nullptr;
    p.nch_magic[0] = g.nch_magic[0];
    p.nch_magic[1] = g.nch_magic[1];
    for (int j = 0; j < 13; j++) p.sin_c[j] = vcrt::kSinC[j];
    const std::array<float, 12> cam = camera_array();
    for (int i = 0; i < 12; i++) p.cam[i] = cam[i];
    const KernelChoice kc = select_kernel();
    hipFunction_t f = g.debug_stats == 1 ? kc.stats : kc.f;
    // Deferred fetches (tracer.hip, the flat scans): the LDS-table flat scan waits until 4 lanes
    // need an item (at most one iteration): C3 -0.6 % kernel time (its 16 items per pixel make
    // the fetch frequent), C4 and the 8-way shards within 0.1 %, same bits; the global-table and
    // boxes-in-LDS scans fetch at once (C5 +0.6 % with it). profiles/r06_ab_log.md.
    const bool lds_flat = kc.f == g.k_trace_cull_flat;
    p.fetch_min = g.fetch_min > 0u ? g.fetch_min : (lds_flat ? 4u : 1u);
    p.fetch_wait = g.fetch_min > 0u ? g.fetch_wait : (lds_flat ? 1u : 0u);
    const uint32_t block = kc.block;
    uint32_t lds = kc.lds;
    // the linear SMEM scan of a small scene stages its shading and jitter tables in LDS
    // (TraceParams.stage_*): C2 (4 spheres, 64 spp) is latency-bound on those reads
    p.stage_spheres = 0u;
    p.stage_spp = 0u;
    if (kc.f == g.k_trace_smem && g.nspheres > 0 && g.stage_tables) {
        // in 64 bits: 16 * spp wraps 32 bits for spp >= 2^28
        const uint64_t bytes = 48ull * static_cast<uint64_t>(g.nspheres) +
                               16ull * static_cast<uint64_t>(g.desc.samples_per_pixel);
        if (bytes <= kStageMaxBytes) {
            p.stage_spheres = static_cast<uint32_t>(g.nspheres);
            p.stage_spp = static_cast<uint32_t>(g.desc.samples_per_pixel);
            lds = static_cast<uint32_t>((bytes + 15u) & ~15ull);
        }
    }
    const int variant = kc.variant;
    // the stage names the entry point this draw dispatches (Shader.cpp:89 names "main")
    g.stage.pName = kc.name;
    std::snprintf(g.stats.kernel, sizeof(g.stats.kernel), "%s%s", kc.name,
                  g.debug_stats == 1 ? "_stats" : "");
    int per_cu = g.desc.blocks_per_cu;
    if (per_cu <= 0) {
        per_cu = 0;
        if (hipModuleOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, f, block, lds) !=
                hipSuccess ||
            per_cu <= 0)
            per_cu = 1;
        if (g.max_blocks_per_cu > 0) per_cu = std::min(per_cu, g.max_blocks_per_cu);
    }
    // Cost order. When the frame gives each lane of the persistent grid few items, its end
    // is set by the last expensive items to start (an item's segments run one per wave
    // iteration: a glass pixel's 16-sample item at depth 8 is ~100 iterations), not by the
    // work. Then the first frame of a configuration counts each pixel's segments
    // (TraceParams.pixel_cost), and later frames hand out the blocks longest items first
    // (TraceParams.block_order, build_block_order); such frames also run at most kDrainWavesPerSimd
    // waves per SIMD, so that the waves holding the last items advance faster. Only the
    // schedule changes: the image depends on the quantum alone. Automatic for the linear
    // scans' frames with few items per lane (C2), and for the cost partition (default_chunk:
    // the 4- and 8-way shards of C4, where the flat scans launch their cost-order builds).
    // Elsewhere the flat scans' static bottom-up order is already roughly cost-ordered (sky
    // last) and keeps neighbouring blocks together: the cost order on their own partitions
    // measured slower (C4 -0.5%, C3 -1.1%, 8-way shards at K = 16 + 128 x 4 -4%;
    // profiles/r05_ab_log.md).
    const uint32_t total_blocks =
        g.local_tiles * static_cast<uint32_t>(g.nchunks + g.tail_nchunks);
    const bool cost_mode =
        g.debug_stats != 1 && total_blocks > 0 && kc.cost != nullptr &&
        (g.cost_order == 1 ||
         (g.cost_order < 0 &&
          (g.cost_partition ||
           (kc.cost == kc.f &&  // (the linear scans)
            static_cast<uint64_t>(g.total_items) <
                kCostOrderItemsPerLane * static_cast<uint64_t>(per_cu) * g.num_cus * block))));
    if (cost_mode && kc.cost != kc.f) {  // the flat scans' cost-order build
        f = kc.cost;
        std::snprintf(g.stats.kernel, sizeof(g.stats.kernel), "%s_cost", kc.name);
    }
    if (cost_mode && g.desc.blocks_per_cu <= 0 && g.max_blocks_per_cu <= 0)
        per_cu = std::min(per_cu, std::max(1, static_cast<int>(kDrainWavesPerSimd * 4u * 64u /
                                                               block)));
    // The accumulation ring (tracer.hip RingEntry): the LDS the workgroups leave free at
    // this occupancy, up to 63 entries of 32 B per wave, when the frame sums chunk sums
    // (not one chunk per pixel), its blocks are chunk-minor and its pixel indices leave the
    // top bits for the entry. The occupancy must not drop for it.
    p.ring_off = 0u;
    p.ring_n = 0u;
    uint32_t lds_launch = lds;
    if (g.accum_ring && !g.direct && (g.work_flags & vcrt::kFlagChunkMinor) != 0u &&
        static_cast<uint64_t>(g.local_tiles) * 64u <= (uint64_t{1} << vcrt::kRingQBits) &&
        g.lds_per_cu > 0 && g.desc.blocks_per_cu <= 0) {
        const uint32_t waves = block / 64u;
        const uint32_t off = (lds + 15u) & ~15u;
        // usable LDS per CU: measured, five 256-thread workgroups of 32512 B ran four per
        // CU (-11% at C4) while 32000 B ran five, although 5 x 32512 < 160 KiB and the
        // occupancy query allows them: budget 160000 B per CU
        const uint32_t per_wg = std::min<uint32_t>(g.lds_per_cu, 160000u) /
                                static_cast<uint32_t>(per_cu);
        uint32_t n = per_wg > off ? std::min<uint32_t>(g.ring_max,
                                                        (per_wg - off) / (32u * waves))
                                  : 0u;
        for (; n >= 8u; n -= 4u) {
            int occ = 0;
            if (hipModuleOccupancyMaxActiveBlocksPerMultiprocessor(
                    &occ, f, block, off + 32u * n * waves) == hipSuccess &&
                occ >= per_cu)
                break;
        }
        if (n >= 8u) {
            p.ring_off = off;
            p.ring_n = n;
            lds_launch = off + 32u * n * waves;
        }
    }
    g.stats.ring_entries = static_cast<int32_t>(p.ring_n);
    const uint32_t grid = static_cast<uint32_t>(per_cu) * static_cast<uint32_t>(g.num_cus);
    const uint64_t key = cost_mode ? order_key_of(kc.f, grid, total_blocks) : 0;
    bool measure = false;
    p.pixel_cost = nullptr;
    p.block_order = nullptr;
    if (cost_mode && key == g.order_key) {
        p.block_order = g.d_block_order;
        p.flags &= ~vcrt::kFlagReverseOrder;  // the order is the whole hand-out sequence
    } else if (cost_mode) {
        if (pixels > g.cost_words) {
            if (g.d_pixel_cost) (void)hipFree(g.d_pixel_cost);
            g.d_pixel_cost = nullptr;
            g.cost_words = 0;
            VCRT_TRY(hipMalloc(&g.d_pixel_cost, pixels * sizeof(uint32_t)));
            g.cost_words = pixels;
        }
        VCRT_TRY(hipMemsetAsync(g.d_pixel_cost, 0, pixels * sizeof(uint32_t), g.stream));
        p.pixel_cost = g.d_pixel_cost;
        measure = true;
    }
    g.stats.cost_order = p.block_order != nullptr ? 1 : 0;
    if (!g.counters_clean) VCRT_TRY(hipMemsetAsync(g.d_counters, 0, kCounterBytes, g.stream));
    g.counters_clean = false;  // until this frame's resolve has read and zeroed them
    if (g.debug_stats == 1) {  // the stats kernels' region counters, one row per wave
        const size_t words = static_cast<size_t>(grid) * (block / 64u) * kRegionCount;
        if (words > g.region_words) {
            if (g.d_region) (void)hipFree(g.d_region);
            g.d_region = nullptr;
            g.region_words = 0;
            VCRT_TRY(hipMalloc(&g.d_region, words * sizeof(uint32_t)));
            g.region_words = words;
        }
        VCRT_TRY(hipMemsetAsync(g.d_region, 0, words * sizeof(uint32_t), g.stream));
        p.region = g.d_region;
    }
    if (!g.direct && !g.desc.progressive && !g.accum_clean)  // every frame sums from zero
        VCRT_TRY(hipMemsetAsync(g.d_accum, 0, 32u * static_cast<size_t>(pixels), g.stream));
    if (!g.direct) g.accum_clean = false;  // until this frame's resolve zeroes it
    if (g.debug_stats) {
        unsigned long long init[128] = {0, 0, 0, 0, 0, ~0ull};
        if (g.debug_stats == 2) init[9] = init[10] = ~0ull;  // wave times: minima
        VCRT_TRY(hipMemcpyAsync(g.d_debug, init, sizeof(init), hipMemcpyHostToDevice,
                                g.stream));
    }
    VCRT_TRY(hipEventRecord(g.ev_start, g.stream));
    VkResult r = launch(f, grid, block, lds_launch, p);
    if (r != VK_SUCCESS) return r;
    VCRT_TRY(hipEventRecord(g.ev_stop, g.stream));
    bool resolved = false;
    if (!g.direct) {
        vcrt::ResolveParams rp{g.d_accum,
                               g.d_fb,
                               std::ldexp(1.0, -g.accum_log2),
                               static_cast<float>(spp_total),
                               g.desc.width,
                               g.desc.height,
                               g.desc.rank,
                               g.desc.world_size,
                               g.tiles_x,
                               g.local_tiles,
                               g.desc.progressive ? 0u : 1u,
                               g.pixel_scale ? g.d_pixel_emax : nullptr,
                               static_cast<unsigned long long*>(g.d_counters),
                               g.h_counters,
                               static_cast<uint32_t>(kCounterBytes / 4)};
        const uint32_t rgrid = std::min<uint32_t>((pixels + 255) / 256, 8192);
        r = launch(g.k_resolve, rgrid, 256, 0, rp);
        if (r != VK_SUCCESS) return r;
        resolved = true;
        g.accum_clean = !g.desc.progressive;
        VCRT_TRY(hipEventRecord(g.ev_resolve, g.stream));
    }
    if (!resolved)  // (one quantum per pixel: no resolve pass)
        VCRT_TRY(hipMemcpyAsync(g.h_counters, g.d_counters, 4 * sizeof(unsigned long long),
                                hipMemcpyDeviceToHost, g.stream));
    VCRT_TRY(hipStreamSynchronize(g.stream));
    g.counters_clean = resolved;
    const unsigned long long* counters = g.h_counters;
    float ms = 0.f;
    VCRT_TRY(hipEventElapsedTime(&ms, g.ev_start, g.ev_stop));
    g.stats.kernel_ms = ms;
    if (!g.direct) {
        VCRT_TRY(hipEventElapsedTime(&ms, g.ev_stop, g.ev_resolve));
        g.stats.resolve_ms = ms;
    }
    g.stats.segments = counters[1];
    g.stats.group_tests = counters[2];
    g.stats.bound_tests = counters[3];
    if (measure) {
        const VkResult ro = build_block_order(total_blocks);
        if (ro != VK_SUCCESS) return ro;
        g.order_key = key;
    }
    if (g.debug_stats)
        VCRT_TRY(hipMemcpy(g.stats.debug, g.d_debug, sizeof(g.stats.debug),
                           hipMemcpyDeviceToHost));
    if (g.debug_stats == 1 && p.region) {  // region counters summed over the waves
        const size_t words = static_cast<size_t>(grid) * (block / 64u) * kRegionCount;
        std::vector<uint32_t> rows(words);
        VCRT_TRY(hipMemcpy(rows.data(), g.d_region, words * sizeof(uint32_t),
                           hipMemcpyDeviceToHost));
        for (size_t w = 0; w < words / kRegionCount; w++)
            for (uint32_t k = 0; k < kRegionCount; k++)
                g.stats.debug[kRegionDebugBase + k] += rows[w * kRegionCount + k];
    }
    g.stats.grid_blocks = static_cast<int32_t>(grid);
    g.stats.block_threads = static_cast<int32_t>(block);
    g.stats.kernel_variant = variant;
    g.stats.lds_bytes = lds;  // tables and stacks; the ring adds ring_entries x 32 B per wave
    g.stats.tables_in_lds = kc.f == g.k_trace_cull_flat_boxes ? 2 :
                            (kc.f == g.k_trace_cull_flat || kc.f == g.k_trace_cull_lane_lds ||
                             kc.f == g.k_trace_cull_lane_lds_wide) ? 1 : 0;
    *outlier_max = static_cast<uint32_t>(counters[0]);
    return VK_SUCCESS;
}

// Outlier quanta (vcrt_math.h "Accumulation"): the render just done saw a quantum sum too large
// for its pixel's scale (every pixel starts at 2^32: |S| >= 2^12). The kernel recorded each such
// pixel's largest |S| in d_pixel_emax; from now on every frame of this configuration quantizes
// each pixel at its own scale, and this frame is rendered again -- a progressive frame together
// with every frame before it, from zero, since their sums were quantized at the old scales. The
// image then depends on each pixel's own samples only (any rank, any schedule). A render at the
// recorded scales sees no outliers (the same samples); a later progressive frame may raise a
// pixel's maximum, and then the same happens again.
static VkResult rerender_scaled(uint64_t spp_total, uint32_t outlier_max) {
    const uint64_t spp = static_cast<uint64_t>(g.desc.samples_per_pixel);
    for (int attempt = 0; outlier_max != 0u; attempt++) {
        if (attempt == 4) return VK_ERROR_UNKNOWN;  // cannot happen: the maxima only grow
        g.pixel_scale = true;
        g.min_scale = std::min(g.min_scale, vcrt::pixel_scale_log2(outlier_max));
        g.stats.accumulate_scale_log2 = g.min_scale;
        g.stats.scale_rerenders += 1;
        outlier_max = 0u;
        if (!g.desc.progressive) {
            VkResult r = trace_frame(spp_total, &outlier_max);
            if (r != VK_SUCCESS) return r;
            continue;
        }
        VCRT_TRY(hipMemsetAsync(g.d_accum, 0, 32u * static_cast<size_t>(g.total_pixels),
                                g.stream));
        for (uint64_t f = 0; f * spp < spp_total; f++) {
            VkResult r = setup_jitter(f * spp);
            if (r == VK_SUCCESS) {
                uint32_t o = 0u;
                r = trace_frame((f + 1) * spp, &o);
                outlier_max = std::max(outlier_max, o);
            }
            if (r != VK_SUCCESS) return r;
        }
    }
    return VK_SUCCESS;
}

vcrt_result vcrt_draw_next_frame(void) {
    if (!g.begun || !g.stage.module) return VCRT_ERROR_INITIALIZATION_FAILED;
    if (g.comm_lost) return VCRT_ERROR_DEVICE_LOST;  // a peer was lost in an earlier frame
    const auto t0 = std::chrono::steady_clock::now();
    const uint32_t pixels = g.total_pixels;
    g.stats.segments = 0;
    g.stats.kernel_ms = 0.0;
    g.stats.resolve_ms = 0.0;
    g.stats.gather_ms = 0.0;
    if (pixels != 0 && g.desc.max_depth == 0) {
        // ray_color with MAX_RECURSION_LEVEL 0 returns its undefined value (canonical 0) for
        // every sample without scanning: the frame is (0,0,0,1).
        vcrt::FillParams fp{g.d_fb, g.local_elems, make_float4(0.f, 0.f, 0.f, 1.f)};
        const uint32_t grid = std::min<uint32_t>((g.local_elems + 255) / 256, 4096);
        VkResult r = launch(g.k_fill, grid, 256, 0, fp);
        if (r != VK_SUCCESS) return r;
    }
    const uint64_t spp_total =
        (g.desc.progressive ? g.accumulated : 0) + static_cast<uint64_t>(g.desc.samples_per_pixel);
    // progressive frames add quanta to the pixels' exact sums: at most kAccumMaxChunks in all
    if (g.desc.progressive &&
        (g.accumulated / static_cast<uint64_t>(g.desc.samples_per_pixel) + 1) *
                static_cast<uint64_t>((g.desc.samples_per_pixel + g.quantum - 1) / g.quantum) >
            static_cast<uint64_t>(vcrt::kAccumMaxChunks))
        return VCRT_ERROR_FORMAT_NOT_SUPPORTED;
    if (g.desc.progressive && g.accumulated > 0) {
        // progressive frames continue the sample sequence: indices accumulated.. (+spp)
        const VkResult rj = setup_jitter(g.accumulated);
        if (rj != VK_SUCCESS) return rj;
    }
    if (pixels != 0 && g.desc.max_depth > 0) {
        g.stats.scale_rerenders = 0;
        uint32_t outlier_max = 0u;
        VkResult r = trace_frame(spp_total, &outlier_max);
        if (r == VK_SUCCESS && outlier_max != 0u) r = rerender_scaled(spp_total, outlier_max);
        if (r != VK_SUCCESS) return r;
    }
    if (g.comm && g.desc.world_size > 1) {
        // this rank's own render is complete (the stream synchronize above, no deadline); the
        // exchange's deadline (wait_gather) scales with the frame time for the peers' renders
        VkResult r = gather_frame();
        if (r == VK_SUCCESS) r = wait_gather();
        if (r != VK_SUCCESS) return r;
        float ms = 0.f;
        VCRT_TRY(hipEventElapsedTime(&ms, g.ev_gather_start, g.ev_gather));
        g.stats.gather_ms = ms;
    }
    VCRT_TRY(hipStreamSynchronize(g.stream));
    g.stats.sphere_tests = g.stats.segments * static_cast<uint64_t>(g.nspheres);
    g.stats.samples =
        static_cast<uint64_t>(g.local_pixels) * static_cast<uint64_t>(g.desc.samples_per_pixel);
    g.stats.frames += 1;
    if (g.desc.progressive && pixels != 0 && g.desc.max_depth > 0)
        g.accumulated += static_cast<uint64_t>(g.desc.samples_per_pixel);
    g.stats.accumulated_spp = g.desc.progressive ? g.accumulated
                                                 : static_cast<uint64_t>(g.desc.samples_per_pixel);
    g.stats.frame_ms =
        std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    return VCRT_SUCCESS;
}

vcrt_result vcrt_end(void) {
    if (!g.begun) return VCRT_SUCCESS;  // idempotent
    if (g.stream) (void)hipStreamSynchronize(g.stream);
    free_scene();
    if (g.d_jitter) (void)hipFree(g.d_jitter);
    if (g.d_jitter_in) (void)hipFree(g.d_jitter_in);
    for (int k = 0; k < 2; k++) {
        if (g.h_jitter[k]) (void)hipHostFree(g.h_jitter[k]);
        if (g.ev_jitter[k]) (void)hipEventDestroy(g.ev_jitter[k]);
    }
    if (g.d_corner) (void)hipFree(g.d_corner);
    if (g.d_fb_own) (void)hipFree(g.d_fb_own);
    if (g.d_counters) (void)hipFree(g.d_counters);
    if (g.h_counters) (void)hipHostFree(g.h_counters);
    if (g.d_debug) (void)hipFree(g.d_debug);
    if (g.d_region) (void)hipFree(g.d_region);
    if (g.d_pixel_cost) (void)hipFree(g.d_pixel_cost);
    if (g.d_block_order) (void)hipFree(g.d_block_order);
    DestroyShaderStage(&g.stage);
    if (g.ev_start) (void)hipEventDestroy(g.ev_start);
    if (g.ev_stop) (void)hipEventDestroy(g.ev_stop);
    if (g.ev_resolve) (void)hipEventDestroy(g.ev_resolve);
    if (g.d_accum) (void)hipFree(g.d_accum);
    if (g.d_pixel_emax) (void)hipFree(g.d_pixel_emax);
    if (g.d_srgb_thresholds) (void)hipFree(g.d_srgb_thresholds);
    if (g.d_srgb) (void)hipFree(g.d_srgb);
    comm_release(false);
    if (g.stream) (void)hipStreamDestroy(g.stream);
    g = RendererState{};
    return VCRT_SUCCESS;
}

vcrt_result vcrt_comm_unique_id(vcrt_comm_id* id) {
    static_assert(sizeof(vcrt_comm_id) == sizeof(ncclUniqueId), "vcrt_comm_id is an ncclUniqueId");
    if (!id) return VCRT_ERROR_INITIALIZATION_FAILED;
    ncclUniqueId u;
    const VkResult r = nccl_vk(ncclGetUniqueId(&u));
    if (r != VK_SUCCESS) return r;
    std::memcpy(id->internal, u.internal, sizeof(u.internal));
    return VCRT_SUCCESS;
}

vcrt_result vcrt_comm_init(const vcrt_comm_id* id) {
    if (!g.begun || !id) return VCRT_ERROR_INITIALIZATION_FAILED;
    if (g.comm) return VCRT_ERROR_INITIALIZATION_FAILED;  // once per vcrt_begin
    VCRT_TRY(hipSetDevice(g.device));  // RCCL binds the communicator to the current device
    VCRT_TRY(hipStreamSynchronize(g.stream));
    ncclUniqueId u;
    std::memcpy(u.internal, id->internal, sizeof(u.internal));
    // non-blocking: set-up and every later operation are waited for with a deadline
    // (comm_wait.hpp), so a rank that never joins fails this call instead of hanging it
    ncclConfig_t config = NCCL_CONFIG_INITIALIZER;
    config.blocking = 0;
    const ncclResult_t e = ncclCommInitRankConfig(&g.comm, g.desc.world_size, u, g.desc.rank,
                                                  &config);
    if (e != ncclSuccess && e != ncclInProgress) {
        if (g.comm) comm_release(true);
        g.comm = nullptr;
        return nccl_vk(e);
    }
    if (vcrt::wait_with_deadline([] { return comm_state(g.comm); }, vcrt::comm_timeout_ms()) !=
        vcrt::WaitResult::kDone) {
        comm_release(true);
        return VCRT_ERROR_INITIALIZATION_FAILED;
    }
    // from here on every failure drops the communicator and the buffers (comm_release)
    auto fail = [](hipError_t err) {
        comm_release(true);
        return to_vk(err);
    };
    hipError_t err;
    if ((err = hipEventCreate(&g.ev_gather_start)) != hipSuccess) return fail(err);
    if ((err = hipEventCreate(&g.ev_gather)) != hipSuccess) return fail(err);
    if (g.desc.world_size > 1 && g.desc.rank == 0) {
        const size_t slab = static_cast<size_t>(g.pad_tiles) * 64 * sizeof(float4);
        const size_t all = slab * static_cast<size_t>(g.desc.world_size);
        if ((err = hipMalloc(&g.d_gather, all)) != hipSuccess) return fail(err);
        if ((err = hipMemsetAsync(g.d_gather, 0, all, g.stream)) != hipSuccess) return fail(err);
        const size_t frame = static_cast<size_t>(g.desc.width) * g.desc.height * sizeof(float4);
        if ((err = hipMalloc(&g.d_frame, frame)) != hipSuccess) return fail(err);
        if ((err = hipMemsetAsync(g.d_frame, 0, frame, g.stream)) != hipSuccess) return fail(err);
        if ((err = hipStreamSynchronize(g.stream)) != hipSuccess) return fail(err);
        g.d_fb = g.d_gather;  // rank 0 renders straight into its slot of the gather buffer
    } else {
        g.d_fb = g.d_fb_own;
    }
    return VCRT_SUCCESS;
}

vcrt_result vcrt_local_layout(uint32_t* elements, uint32_t* tiles) {
    if (!g.begun || !elements || !tiles) return VCRT_ERROR_INITIALIZATION_FAILED;
    *elements = fb_view().elems;
    *tiles = g.local_tiles;
    return VCRT_SUCCESS;
}

vcrt_result vcrt_read_framebuffer(float* rgba, size_t count) {
    const FbView v = fb_view();
    const size_t bytes = static_cast<size_t>(v.elems) * sizeof(float4);
    if (!g.begun || (!rgba && bytes)) return VCRT_ERROR_INITIALIZATION_FAILED;
    if (count * sizeof(float) < bytes) return VCRT_ERROR_FORMAT_NOT_SUPPORTED;
    if (bytes) VCRT_TRY(hipMemcpy(rgba, v.ptr, bytes, hipMemcpyDeviceToHost));
    return VCRT_SUCCESS;
}

vcrt_result vcrt_framebuffer_device(void** device_ptr, size_t* bytes) {
    if (!g.begun || !device_ptr || !bytes) return VCRT_ERROR_INITIALIZATION_FAILED;
    const FbView v = fb_view();
    *device_ptr = v.ptr;
    *bytes = static_cast<size_t>(v.elems) * sizeof(float4);
    return VCRT_SUCCESS;
}

vcrt_result vcrt_set_framebuffer_device(void* device_ptr, size_t bytes) {
    if (!g.begun) return VCRT_ERROR_INITIALIZATION_FAILED;
    if (g.comm) return VCRT_ERROR_FEATURE_NOT_PRESENT;  // the gather owns the buffers
    if (device_ptr == nullptr) {
        g.d_fb = g.d_fb_own;
        return VCRT_SUCCESS;
    }
    if (bytes < g.fb_bytes || (reinterpret_cast<uintptr_t>(device_ptr) & 15u))
        return VCRT_ERROR_FORMAT_NOT_SUPPORTED;
    g.d_fb = static_cast<float4*>(device_ptr);
    return VCRT_SUCCESS;
}

vcrt_result vcrt_assemble_tiles(const void* gathered, void* frame, int32_t width,
                                int32_t height, int32_t world_size, uint32_t tiles_per_rank) {
    if (!g.begun || !gathered || !frame) return VCRT_ERROR_INITIALIZATION_FAILED;
    if (width <= 0 || height <= 0 || world_size <= 0) return VCRT_ERROR_INITIALIZATION_FAILED;
    for (int32_t r = 0; r < world_size; r++)  // every rank's tiles must fit its slab
        if (tiles_for_rank(width, height, world_size, r) > tiles_per_rank)
            return VCRT_ERROR_FORMAT_NOT_SUPPORTED;
    vcrt::AssembleParams ap{static_cast<const float4*>(gathered),
                            static_cast<float4*>(frame),
                            width,
                            height,
                            world_size,
                            static_cast<uint32_t>((width + 7) / 8),
                            tiles_per_rank};
    const uint64_t total = static_cast<uint64_t>(width) * height;
    const uint32_t grid = static_cast<uint32_t>(std::min<uint64_t>((total + 255) / 256, 8192));
    VkResult r = launch(g.k_assemble, grid, 256, 0, ap);
    if (r != VK_SUCCESS) return r;
    VCRT_TRY(hipStreamSynchronize(g.stream));
    return VCRT_SUCCESS;
}

vcrt_result vcrt_reset_accumulation(void) {
    if (!g.begun) return VCRT_ERROR_INITIALIZATION_FAILED;
    VCRT_TRY(hipStreamSynchronize(g.stream));
    VCRT_TRY(reset_sums());
    g.accumulated = 0;
    return setup_jitter(0);
}

vcrt_result vcrt_selftest_sin(uint32_t first, uint32_t count, uint64_t* mismatches,
                              uint64_t* fallbacks, uint32_t* first_mismatch) {
    if (!g.begun || !mismatches || !fallbacks || !first_mismatch)
        return VCRT_ERROR_INITIALIZATION_FAILED;
    hipFunction_t f = nullptr;
    VCRT_TRY(hipModuleGetFunction(&f, static_cast<hipModule_t>(g.stage.module), "vcrt_check_sin"));
    void* buf = nullptr;  // [2] counters + first mismatch
    VCRT_TRY(hipMalloc(&buf, 24));
    uint32_t init[6] = {0, 0, 0, 0, 0xFFFFFFFFu, 0};
    hipError_t e = hipMemcpy(buf, init, sizeof(init), hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipStreamSynchronize(nullptr);  // (the check runs on g.stream)
    vcrt::SinCheckParams sp{static_cast<unsigned long long*>(buf),
                            reinterpret_cast<uint32_t*>(static_cast<char*>(buf) + 16), first, count,
                            {}};
    for (int j = 0; j < 13; j++) sp.sin_c[j] = vcrt::kSinC[j];
    VkResult r = e == hipSuccess ? launch(f, 8 * 256 * 8, 256, 0, sp) : to_vk(e);
    uint32_t out[6] = {0, 0, 0, 0, 0, 0};
    if (r == VK_SUCCESS) {
        e = hipMemcpyAsync(out, buf, sizeof(out), hipMemcpyDeviceToHost, g.stream);
        if (e == hipSuccess) e = hipStreamSynchronize(g.stream);
        r = to_vk(e);
    }
    (void)hipFree(buf);
    if (r != VK_SUCCESS) return r;
    std::memcpy(mismatches, &out[0], 8);
    std::memcpy(fallbacks, &out[2], 8);
    *first_mismatch = out[4];
    return VCRT_SUCCESS;
}

vcrt_result vcrt_read_framebuffer_srgb8(uint8_t* rgba8, size_t bytes) {
    const FbView v = fb_view();
    if (!g.begun || (!rgba8 && v.elems)) return VCRT_ERROR_INITIALIZATION_FAILED;
    if (bytes < static_cast<size_t>(v.elems) * 4) return VCRT_ERROR_FORMAT_NOT_SUPPORTED;
    if (!v.elems) return VCRT_SUCCESS;
    if (g.d_srgb) (void)hipFree(g.d_srgb);  // the view may have grown (vcrt_comm_init)
    g.d_srgb = nullptr;
    VCRT_TRY(hipMalloc(&g.d_srgb, sizeof(uchar4) * v.elems));
    vcrt::EncodeParams ep{v.ptr, g.d_srgb, g.d_srgb_thresholds, v.elems};
    const uint32_t grid = std::min<uint32_t>((v.elems + 255) / 256, 4096);
    VkResult r = launch(g.k_encode, grid, 256, 0, ep);
    if (r != VK_SUCCESS) return r;
    VCRT_TRY(hipMemcpyAsync(rgba8, g.d_srgb, sizeof(uchar4) * v.elems,
                            hipMemcpyDeviceToHost, g.stream));
    VCRT_TRY(hipStreamSynchronize(g.stream));
    return VCRT_SUCCESS;
}

void vcrt_srgb8_thresholds(float thresholds[255]) {
    if (thresholds) srgb_thresholds(thresholds);
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
    const VkResult r = load_code_object(filename);
    if (r == VK_SUCCESS && g.d_geom) g.stage.pName = select_kernel().name;
    return r;
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

int32_t vcrt_cull_tables(const vcrt_sphere* spheres, int32_t count, float* geom, float* bound,
                         float* node, float* top, int32_t* index, int32_t* big_groups,
                         float* margin4, int32_t cap_groups) {
    if (count < 0 || (count > 0 && !spheres)) return 0;
    vcrt::CullTables ct;
    if (!vcrt::build_cull_tables(spheres, count, ct)) return 0;
    if (big_groups) *big_groups = ct.nbig;
    if (margin4) std::memcpy(margin4, ct.margin, sizeof(ct.margin));
    if (ct.nbig + ct.ngroups <= cap_groups) {
        if (geom) std::memcpy(geom, ct.geom.data(), sizeof(float) * ct.geom.size());
        if (bound) std::memcpy(bound, ct.bound.data(), sizeof(float) * ct.bound.size());
        if (node) std::memcpy(node, ct.node.data(), sizeof(float) * ct.node.size());
        if (top) std::memcpy(top, ct.top.data(), sizeof(float) * ct.top.size());
        if (index) std::memcpy(index, ct.index.data(), sizeof(int32_t) * ct.index.size());
    }
    return ct.ngroups;
}

namespace {
// Culling tables and the kernels' camera array for a desc (host only).
bool host_camera_tables(const vcrt_sphere* spheres, int32_t count, const vcrt_render_desc* desc,
                        vcrt::CullTables& ct, float cam[12]) {
    if (!desc || !desc_valid(*desc) || count < 0 || (count > 0 && !spheres)) return false;
    if (!vcrt::build_cull_tables(spheres, count, ct)) return false;
    const vcrt_camera& c = desc->camera;
    const vcrt::Camera cm = vcrt::make_camera(desc->width, desc->height,
                                              vcrt::mk(c.lookfrom[0], c.lookfrom[1], c.lookfrom[2]),
                                              vcrt::mk(c.lookat[0], c.lookat[1], c.lookat[2]),
                                              vcrt::mk(c.vup[0], c.vup[1], c.vup[2]), c.vfov,
                                              [](double x) { return std::tan(x); });
    const vcrt::f3 v[4] = {cm.pixel00, cm.delta_u, cm.delta_v, cm.center};
    for (int i = 0; i < 4; i++) {
        cam[3 * i + 0] = v[i].x;
        cam[3 * i + 1] = v[i].y;
        cam[3 * i + 2] = v[i].z;
    }
    return true;
}
}  // namespace

int32_t vcrt_primary_lists(const vcrt_sphere* spheres, int32_t count, const vcrt_render_desc* desc,
                           uint32_t* info, int32_t cap_tiles, uint16_t* ids, int32_t cap_ids) {
    vcrt::CullTables ct;
    float cam[12];
    if (!host_camera_tables(spheres, count, desc, ct, cam)) return -1;
    vcrt::PrimaryLists pl;
    vcrt::build_primary_lists(ct, cam, desc->width, desc->height, desc->rank, desc->world_size,
                              pl);
    if (info && cap_tiles >= static_cast<int32_t>(pl.info.size()))
        std::memcpy(info, pl.info.data(), sizeof(uint32_t) * pl.info.size());
    if (ids && cap_ids >= static_cast<int32_t>(pl.ids.size()))
        std::memcpy(ids, pl.ids.data(), sizeof(uint16_t) * pl.ids.size());
    return static_cast<int32_t>(pl.ids.size());
}

int32_t vcrt_primary_sphere_lists(const vcrt_sphere* spheres, int32_t count,
                                  const vcrt_render_desc* desc, uint32_t* info, int32_t cap_tiles,
                                  float* rec, int32_t cap_floats) {
    vcrt::CullTables ct;
    float cam[12];
    if (!host_camera_tables(spheres, count, desc, ct, cam)) return -1;
    vcrt::PrimarySphereLists sl;
    vcrt::build_primary_sphere_lists(ct, spheres, cam, desc->width, desc->height, desc->rank,
                                     desc->world_size, sl);
    if (info && cap_tiles >= static_cast<int32_t>(sl.info.size()))
        std::memcpy(info, sl.info.data(), sizeof(uint32_t) * sl.info.size());
    if (rec && cap_floats >= static_cast<int32_t>(sl.rec.size()))
        std::memcpy(rec, sl.rec.data(), sizeof(float) * sl.rec.size());
    return static_cast<int32_t>(sl.rec.size() / 12);
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
