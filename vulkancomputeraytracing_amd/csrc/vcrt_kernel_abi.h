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

// The frame is cut into 8x8 pixel tiles (tx, ty). Rank r of world owns the tiles with
// (tx + ty) % world == r, numbered row-major as local tiles lt (vcrt_math.h tile_of /
// owner_of). Work items are (local tile, sample
// chunk, slot): 64 consecutive items are one tile at one chunk of samples, one lane per pixel.
// Rank-local framebuffer: world == 1 -> the frame itself, row-major [H][W]; world > 1 -> packed
// tiles [local_tiles][64] (slot = 8 * (y % 8) + x % 8), re-interleaved by vcrt_assemble.
struct TraceParams {
    const float4* geom;           // pair-SoA sphere groups (+1 padding group), scan input
    const float4* center_radius;  // [n] (center.xyz, radius)           -- read once per hit
    const float4* shade;          // [n] (colour.rgb, texture.y = param)
    const float4* material;       // [n] (texture.x = material id, 1 / texture.y, Schlick r0^2
                                  //   of texture.y, 0): the glass quotients precomputed (fp32)
    // shader.comp:43-49's viewport point pixel00 + x delta_u + y delta_v + jx delta_u + jy delta_v
    // is the sum of two fp32 terms: the pixel's corner (the `corner` table below for the culled
    // scans, computed at each sample start by the linear ones) and the sample's jitter term, a
    // table (vcrt_setup_jitter, the kernel's own operations)
    const float4* jitter;  // [spp] jx delta_u + jy delta_v, (jx, jy) = (-0.5+rand(i,i),
                           //   -0.5+rand(i+1,i+1)) of sample index i (shader.comp:48)
    float4* out;           // rank-local framebuffer, rgba32f (layout above)
    double* accum;         // [local_tiles * 64][4] exact sums of the quantized quantum sums (r,
                           //   g, b, unused), vcrt_math.h "Accumulation"; unused with kFlagDirect
    uint32_t* work;        // eight work-queue counters kQueueStride apart, zeroed every launch
    unsigned long long* segments;  // ray segments traced, zeroed before every launch
    unsigned long long* debug;     // diagnostics counters (stats kernels only), may be null
    unsigned long long* work_done;  // [2]: sphere groups tested, group bounds tested
    // spatially clustered copy of the scene for the culled scan (kernel variant CULL)
    const float4* cgroup;   // [(nbig + ncgroups) * 5] per group: four pair-SoA float4s
                            //   (cx0,cx1,cy0,cy1) (cz0,cz1,r0^2,r1^2) (cx2..) (cz2..) + the
                            //   members' world[] indices as int bits (-1 = padding); the nbig
                            //   big-sphere groups first, then the hierarchy in spatial order
    const float4* cbound;   // [ncgroups / 2 * 4] boxes of group pairs, pair-SoA:
                            //   (lox0,lox1,loy0,loy1) (loz0,loz1,hix0,hix1) (hiy0,hiy1,hiz0,hiz1)
                            //   (K0,K1,0,0), K = 8.1u / r_min of the box's members
    const float4* cbound_nf;  // [ncgroups / 2 * 5] the same group-pair boxes for the flat
                              //   scan's near/far reads: per axis (lo0,lo1,hi0,hi1,lo0,lo1),
                              //   x then y then z, then (K0,K1) -- 80 B per pair
    const float4* cnode;    // [ncgroups / 16 * 4] boxes of node pairs (8 groups per node)
    const float4* ctop;     // boxes of pairs of 64-group chunks, same form
    const float4* cnode_nf;  // [ceil(ncgroups / 64) * 4 * 5] the node-pair boxes in the near/far
                             //   layout of cbound_nf, padded to whole chunks (the flat scan's
                             //   chunk passes)
    const uint32_t* prim_info;  // [4 local_tiles][2] camera-ray lists of each 4x4 quarter
                                //   (4 lt + 2 qy + qx) of each local tile, or null: [0] the
                                //   hierarchy groups (main scan) as offset << 4 | count (<= 8),
                                //   [1] the spheres (camera fast trace) as first pair << 4 |
                                //   count (<= 14); 15 = no list
    const uint16_t* prim_ids;   // hierarchy group indices of the group lists
    const float4* cam_rec;      // with the lists: [nbig * 4] the big groups' camera-relative
                                //   records, pair-SoA (ocx0,ocx1,ocy0,ocy1) (ocz0,ocz1,cc0,cc1)
                                //   (..2,3..) with oc = camera centre - centre, cc = |oc|^2 - r^2,
                                //   fp32 as pair_disc_cc computes them; then the sphere lists'
                                //   pair records [pairs * 3]: (ocx0,ocx1,ocy0,ocy1)
                                //   (ocz0,ocz1,cc0,cc1) (index0, index1 as int bits, 0, 0)
                                //   (cluster.hpp build_camera_records / build_primary_sphere_lists)
    float box_margin[4];    // max |centre|, r_max^2, max |box coordinate|, 0 (rounded up)
    int32_t ncgroups;       // hierarchy groups, multiple of 16
    int32_t nbig;           // big-sphere groups tested for every ray
    int32_t nspheres;
    int32_t width, height, spp, max_depth;
    int32_t rank, world;
    uint32_t tiles_x;      // ceil(width / 8)
    uint32_t local_tiles;  // tiles owned by this rank
    uint32_t total_items;  // local_tiles * 64 * (nchunks + tail_nchunks)
    int32_t chunk;         // samples per work item (<= kAccumMaxChunk) of the head
    int32_t nchunks;       // ceil(tail_start / chunk)
    // The tail: samples tail_start .. spp-1 of every pixel in chunks of tail_chunk (tail_nchunks
    // of them), handed out after all head blocks (the first blocks_head = local_tiles *
    // nchunks). No tail: tail_start = spp, tail_nchunks = 0.
    int32_t tail_start, tail_chunk, tail_nchunks;
    uint32_t blocks_head;
    // the accumulation quantum G - 1 (G a power of two): a lane's fp32 sum is quantized and added
    // to the pixel's sums at every sample index that is a multiple of G (vcrt_math.h
    // "Accumulation"); items hold whole quanta
    uint32_t quantum_mask;
    uint32_t flags;        // kFlag*; bits 24..31: s + 128, the quantization scale 2^s every
                           //   pixel's quantum sums start at (vcrt_math.h "Accumulation":
                           //   2^32; kFlagPixelScale: each pixel's own from pixel_emax), kept in
                           //   the flags word the retire reads anyway (no load of its own)
    float spp_total;       // kFlagDirect: the divisor (samples per pixel)
    float cam[12];         // pixel00.xyz, delta_u.xyz, delta_v.xyz, center.xyz
    // Per-wave accumulation ring in LDS (tracer.hip "Accumulation ring"): ring_n entries of 32 B
    // per wave (0: none; <= kRingMaxEntries) at byte ring_off of the dynamic LDS, wave w of the
    // workgroup at ring_off + 32 ring_n w. Needs local pixels < 2^kRingQBits.
    uint32_t ring_off, ring_n;
    // The linear SMEM scan's staging (small scenes, C2): when stage_spp != 0 the kernel copies
    // the shading tables of the stage_spheres spheres (center_radius, shade, material: 48 B each)
    // and the jitter table (stage_spp float4) to the start of the dynamic LDS and reads them
    // there: the per-hit and per-sample reads leave global memory (L2 latency on every bounce).
    uint32_t stage_spheres, stage_spp;
    double sin_c[13];  // vcrt_math.h kSinC: the fast sine's constants, read by scalar loads
    const float4* corner;  // [local_tiles * 64] pixel00 + x delta_u + y delta_v per local slot
                           //   (shader.comp:43; vcrt_setup_jitter, the kernel's own operations)
    // chunk-minor slots: (i * nch_magic[part]) >> 32 = i / nchunks of the head (0) / the tail (1)
    // for every item index i < 64 nchunks (host-checked; 0: the kernel divides)
    uint32_t nch_magic[2];
    // deferred fetches (the flat scans): a wave whose lanes still have work fetches items only
    // once fetch_min lanes need one or it has deferred fetch_wait iterations (1, 0: every time)
    uint32_t fetch_min, fetch_wait;
    // stats builds only (VCRT_DEBUG_STATS=1): [waves][88] region entry counts (tracer.hip
    // reg::*), zeroed before the launch; null otherwise
    uint32_t* region;
    // the cost-ordered schedule (drain-bound frames, capi.cpp "cost order"): pixel_cost, when
    // set, receives each local pixel's segments (u32, modular: an item subtracts the lane's
    // segment count at its start and adds it at its end); block_order, when set, maps the k-th
    // block a part hands out to the block of that part to run (the reverse flag is then off)
    uint32_t* pixel_cost;
    const uint32_t* block_order;
    // Outlier quanta (vcrt_math.h "Accumulation"): a quantum sum with |S * 2^s| >= 2^44 (finite)
    // atomicMax-es the float bits of its largest |channel| into pixel_emax[local pixel] and into
    // *outlier_max; with kFlagPixelScale every pixel quantizes at pixel_scale_log2(pixel_emax[.])
    // instead of the flags' scale
    uint32_t* pixel_emax;
    uint32_t* outlier_max;
};

constexpr uint32_t kQueueStride = 32;  // u32s between the work-queue counters (128 B)
#ifndef VCRT_QUEUES
#define VCRT_QUEUES 32
#endif
// work queues (a power of two): queue x serves workgroups x, x + kQueues, ..., which all sit
// on XCD x % 8; 32 (four per XCD) measured at or above 8 and 16 (profiles/r03_ab_log.md)
constexpr uint32_t kQueues = VCRT_QUEUES;
constexpr uint32_t kMaxQueues = 32;        // counters the host allocates and zeroes
constexpr uint32_t kRingMaxEntries = 63;  // entry + 1 in the top 6 bits of a lane's pixel index
constexpr uint32_t kRingQBits = 26;
// the kernel masks a queue index with kQueues - 1 and the host zeroes kMaxQueues counters
static_assert((kQueues & (kQueues - 1u)) == 0u && kQueues >= 1u && kQueues <= kMaxQueues,
              "VCRT_QUEUES: a power of two <= kMaxQueues");
static_assert(kRingMaxEntries + 1u <= (1u << (32u - kRingQBits)), "ring entry field");

constexpr int32_t kFlatMaxGroups = 1024;   // CULL_FLAT 16-bit entries: 10-bit group / node fields
constexpr int32_t kFlatMaxGroups8 = 256;   // the LDS-table kernel: 8-bit fields, 16-bit candidates
constexpr uint32_t kWaveScratchBytes = 4360;   // CULL_FLAT per-wave LDS stacks, 16-bit entries
constexpr uint32_t kWaveScratchBytes8 = 3464;  // 16-bit candidates, no chunk stack (LDS tables)
constexpr uint32_t kWaveScratchBytesWide = 6920;  // the same with 32-bit entries (global tables)
constexpr uint32_t kFlagReverseOrder = 1u;  // hand out work items last-to-first
constexpr uint32_t kFlagSceneBounded = 2u;  // every |center|, radius <= 2^30 (host-checked)
constexpr uint32_t kFlagChunkMinor = 8u;  // a block's 64 items run chunk-minor: all chunks of
                                          // 64 / nchunks pixels (else one chunk of 64 pixels)
constexpr uint32_t kFlagRadiiSafe = 16u;  // every |radius| in [2^-40, 2^30] (host-checked):
                                         // shading's (p - c) / r may take the unscaled division
constexpr uint32_t kFlagScaleShift = 24u;  // TraceParams.flags: s + kFlagScaleBias
constexpr int32_t kFlagScaleBias = 128;
constexpr uint32_t kFlagPixelScale = 32u;  // per-pixel scales from TraceParams.pixel_emax
constexpr uint32_t kFlagDirect = 4u;  // one work item per pixel and frame, not progressive: the
                                      // lane writes the pixel itself (no sums, no resolve pass)

// TraceParams.jitter from the host's jitter (vcrt_math.h rand2) and the camera: run at
// vcrt_begin and for each progressive frame.
struct SetupJitterParams {
    const float2* jitter_in;  // [nsamples] (jx, jy)
    float4* jitter;           // [nsamples] jx delta_u + jy delta_v
    uint32_t nsamples;
    float cam[12];  // as TraceParams.cam
    float4* corner;  // [slots] the local slots' pixel corners, or null
    uint32_t slots, tiles_x, rank, world;
};

// Exact sums -> pixels (vcrt_math.h resolve_channel), rgba32f with alpha 1.
struct ResolveParams {
    double* accum;                    // [local_tiles * 64][4]
    float4* out;                      // rank-local framebuffer
    double inv_scale;                 // 2^-s (the scale of TraceParams.flags bits 24..31)
    float spp_total;                  // samples per pixel accumulated so far (<= 2^19)
    int32_t width, height, rank, world;
    uint32_t tiles_x, local_tiles;
    uint32_t zero_accum;  // 1: write zeros back (the next frame sums from zero: no memset)
    const uint32_t* pixel_emax;  // non-null: each pixel's own scale (vcrt_math.h pixel_scale_log2)
    // the tracer's counters (TraceParams outlier_max, segments, work_done, work queues), or
    // null: block 0 copies their first four u64 to counters_out (host-pinned) and then zeroes
    // counter_words u32 of them, so the next frame needs neither a memset nor a read-back copy
    unsigned long long* counters;
    unsigned long long* counters_out;
    uint32_t counter_words;
};

struct AssembleParams {
    const float4* gathered;  // [world][tiles_per_rank][64] packed rank framebuffers
    float4* frame;           // [height][width]
    int32_t width, height, world;
    uint32_t tiles_x, tiles_per_rank;
};

// Linear rgba32f -> sRGB8 as the reference's B8G8R8A8_SRGB swapchain stores it (Frontend.cpp:43).
struct EncodeParams {
    const float4* in;
    uchar4* out;
    const float* thresholds;  // [255] ascending: byte = #{k : c >= thresholds[k]}
    uint32_t count;
};

struct SinCheckParams {
    unsigned long long* result;  // [2]: inputs where sin_fast != sin_canonical, fallbacks
    uint32_t* first_bad;         // smallest differing bit pattern (init 0xFFFFFFFF)
    uint32_t first, count;       // input bit patterns first .. first + count - 1
    double sin_c[13];            // vcrt_math.h kSinC, for the table form the tracer uses
};

struct FillParams {
    float4* out;
    uint32_t count;
    float4 value;
};

}  // namespace vcrt
