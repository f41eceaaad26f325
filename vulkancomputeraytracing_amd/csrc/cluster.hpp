// cluster.hpp -- spatial grouping of the sphere list for the culled scan (variant CULL).
//
// The reference scans world[] linearly for every ray (functions.glsl:77-81). Because that scan
// picks the smallest accepted t with ties to the earliest index (tracer.hip, scan_culled), the
// spheres can be visited in any order; this module reorders them into spatially compact groups
// of four with conservative axis-aligned boxes so a wave can skip groups no lane's ray comes
// near.
#pragma once

#include <cstdint>
#include <vector>

#include "vcrt.h"

namespace vcrt {

constexpr int kNodeGroups = 8;  // groups per node of the box hierarchy
constexpr size_t kFlatGroups16 = 1024;  // = vcrt::kFlatMaxGroups (10-bit entry fields)

struct CullTables {
    int32_t nbig = 0;             // big-sphere groups, first in geom/index, tested for every ray
    int32_t ngroups = 0;          // hierarchy groups after them, a multiple of 2 * kNodeGroups
    std::vector<float> geom;      // [nbig + ngroups][16] pair-SoA, same values as the linear table
    std::vector<int32_t> index;   // [nbig + ngroups][4] world[] index of each member, -1 = padding
    std::vector<float> bound;     // [ngroups / 2][16] hierarchy group-pair boxes (TraceParams)
    std::vector<float> node;      // [ngroups / kNodeGroups / 2][16] node-pair boxes, same form
    std::vector<float> top;       // [ceil(ngroups / 64) rounded up to even / 2][16] boxes of
                                  // each 64-group chunk (8 nodes), same form
    float margin[4] = {0, 0, 0, 0};  // box-test constants over the hierarchy: max |centre|,
                                     // r_max^2, max |coordinate| of a box (rounded up), 0
};

// Builds the grouped tables. Returns false (tables empty) when culling does not apply: fewer
// than 16 spheres or any centre/radius outside +-2^30 (or not finite).
bool build_cull_tables(const vcrt_sphere* spheres, int32_t count, CullTables& out);

// Primary-ray lists (the flat scan's camera rays skip the node level): for every 4x4-pixel
// quarter of every local 8x8 tile, the hierarchy groups a camera ray through it may need, by a
// conservative pyramid-box test in double (primary.cpp). info[4 lt + 2 qy + qx] =
// offset << 4 | count, count <= 8, or kPrimaryNone (those camera rays take the hierarchy).
constexpr uint32_t kPrimaryMax = 8;
constexpr uint32_t kPrimaryNone = 15;

struct PrimaryLists {
    std::vector<uint32_t> info;  // [4 x local tiles]
    std::vector<uint16_t> ids;   // hierarchy group indices, by tile
};

// cam: pixel00, delta_u, delta_v, centre (shader.comp:18-43) as the kernels get them.
void build_primary_lists(const CullTables& ct, const float cam[12], int32_t width,
                         int32_t height, int32_t rank, int32_t world, PrimaryLists& out);

// Per-sphere camera lists (round 3) for the camera fast trace: for every 4x4-pixel quarter of
// every local tile, the hierarchy's spheres a camera ray through it may need (the members of its
// group list whose sphere, grown by its own margin M_s = 8.1u (|oc|^2 + r^2) / r and 1e-3, no
// side plane of the quarter's pyramid separates: primary.cpp), as camera-relative pair records:
// per pair of spheres (ocx0,ocx1,ocy0,ocy1) (ocz0,ocz1,cc0,cc1) (index0,index1 as int bits,0,0),
// evaluated as pair_disc_cc would (an odd count pads its last pair with oc = 0, cc = 3e38, index
// -1: never a candidate). info[4 lt + 2 qy + qx] = first pair << 4 | spheres (<= 14), or
// kPrimaryNone. On average ~1.1 spheres per quarter at the final scene's 1080p camera, against
// ~10.6 members of the listed groups.
constexpr uint32_t kPrimarySphereMax = 14;

struct PrimarySphereLists {
    std::vector<uint32_t> info;  // [4 x local tiles]
    std::vector<float> rec;      // [pairs][12]
};

void build_primary_sphere_lists(const CullTables& ct, const vcrt_sphere* spheres,
                                const float cam[12], int32_t width, int32_t height, int32_t rank,
                                int32_t world, PrimarySphereLists& out);

// Camera-relative group records for the camera fast trace: for every group of ct.geom (big
// groups first), the members' oc = camera centre - centre and cc = |oc|^2 - r^2 in the group
// record's pair-SoA form, (ocx0,ocx1,ocy0,ocy1) (ocz0,ocz1,cc0,cc1) per pair, evaluated in fp32
// with the kernel's operations and order (tracer.hip pair_disc_cc), so a camera ray's hb and
// discriminant from them carry the same bits. [nbig + ngroups][16] floats.
void build_camera_records(const CullTables& ct, const float cam[12], std::vector<float>& out);

}  // namespace vcrt
