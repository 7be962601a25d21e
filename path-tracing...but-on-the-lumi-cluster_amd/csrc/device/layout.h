// Device-side data layout in HBM (shared by the HIP kernels and the host
// code that packs it).  See DESIGN.md "Data layout in HBM".
//
// The reference arrays are repacked once into records a walk step reads
// with independent 16-byte loads:
//   BlockCopy 128 B  4-wide BVH blocks of both levels (block_format.h), one
//                    copy per octant: one 112-byte read per step.
//   TriRec    48 B  the three vertex positions of triangle t of a mesh,
//                   tris[index_offset/3 + t] (ray_query.hh:228-234 gathers
//                   indices then positions: two dependent loads -> one).
//   InstTrav  64 B  what ray_query_enter_blas needs (ray_query.hh:153-182):
//                   inv_transform rows 0..3 (xyz), with the BLAS root block
//                   and the mesh's triangle base in w.
//   InstShade 64 B  what the closest-hit shading needs (path_tracer.hh:369-392):
//                   transform rows 0..2 xyz and the mesh offsets.
// BLAS blocks are packed once (when an instance first names the BLAS); the
// frame's TLAS blocks follow them in the same buffer.
#pragma once
#include <stdint.h>
#include "block_format.h"

namespace ptg {

struct alignas(16) TriRec {
    float p0x, p0y, p0z, p1x;
    float p1y, p1z, p2x, p2y;
    float p2z, pad0, pad1, pad2;
};
static_assert(sizeof(TriRec) == 48, "TriRec is three 16-byte loads");

// TriShade 128 B: what the shading of a hit on triangle t of a mesh reads
// (path_tracer.hh:373-392: three indices, then each vertex's normal, albedo
// and material), gathered once per mesh at tri_shade[index_offset/3 + t]:
// vertex k's normal xyz, albedo xyz and material xyzw at floats 10k..10k+9,
// then 2 pad floats - eight 16-byte loads of one 128-byte line instead of
// three index loads and nine dependent gathers.
struct alignas(16) TriShade {
    float v[32];
};
static_assert(sizeof(TriShade) == 128, "TriShade is one 128-byte line");

struct alignas(16) InstTrav {
    // row k = inv_transform.r[k].{x,y,z} in xyz; w = the BLAS's root block,
    // the mesh's triangle base, 0, 0 for rows 0..3: four whole, aligned
    // 16-byte loads
    float4 row[4];
};
static_assert(sizeof(InstTrav) == 64, "InstTrav is four 16-byte loads");

struct alignas(16) InstShade {
    float rot[9];              // transform.r[k].{x,y,z} for k = 0..2
    uint32_t index_offset, base_vertex_offset, pad[5];
};
static_assert(sizeof(InstShade) == 64, "InstShade is four 16-byte loads");

// InstBox 32 B: an instance's TLAS leaf box (the reference's leaf node, the
// bounds of its transformed BLAS root box, bvh.cc:259-281) and where it is a
// leaf: the any-hit walk's occluder candidates (k_wf_walk<ANY>) test an
// instance's leaf box directly, without walking the TLAS down to it.
//   lo.xyz, w = sub: the one subframe whose TLAS holds the instance, or
//                    kInstAllSubframes (every TLAS holds it, with this same box),
//                    or kInstNoCandidate (neither: never a candidate)
//   hi.xyz, w = the triangle count of its mesh (candidate triangles are below it)
struct alignas(16) InstBox {
    float lo[3];
    uint32_t sub;
    float hi[3];
    uint32_t tri_count;
};
static_assert(sizeof(InstBox) == 32, "InstBox is two 16-byte loads");
constexpr uint32_t kInstAllSubframes = 0xFFFFFFFFu, kInstNoCandidate = 0xFFFFFFFEu;

// Everything a hot-path kernel reads, passed by value as a kernel argument.
struct DevScene {
    const BlockCopy* blocks;       // block BVH records of both levels (block_format.h), 8 copies per block
    const uint32_t* tlas_root;     // per subframe: its TLAS's root block
    const TriRec* tris;
    const TriShade* tri_shade;     // per mesh triangle, at the TriRec's index
    const InstTrav* inst_trav;
    const InstShade* inst_shade;
    const InstBox* inst_box;       // per instance: TLAS leaf box + membership (occluder candidates)
    const uint32_t* indices;
    const float* normal;           // reference float3[] (16 B stride)
    const float* albedo;           // float4[]
    const float* material;         // float4[]
    const uint8_t* subframes;      // reference subframe[] (160 B each)
    const float2* polygon;         // per subframe: (sin, cos) of the aperture polygon's vertex angles (kPolyStride each)
    uint32_t width, height, spp, max_bounces, student_id, blur_step;
    uint32_t subframe_count;
    // bounds of the record buffers, checked only by PTG_DEBUG builds
    uint32_t block_count, tri_count, inst_count;
    uint2* spill;                  // LdsStack spill areas, spill_stride entries per walk lane
    uint32_t spill_stride;
    uint32_t* debug;               // PTG_DEBUG: violation counters (kDebug* slots), else null
    uint32_t attrs_finite;         // every vertex albedo / material value finite (last_bounce_moot)
};

// PTG_DEBUG builds check every index the walks and the shading derive from
// the records before they use it; a violation is counted in DevScene::debug
// (slot below), the walk of that ray ends instead of reading out of bounds,
// and the render returns PTG_E_RANGE naming the slot.
#ifndef PTG_DEBUG
#define PTG_DEBUG 0
#endif
enum : uint32_t { kDebugNode = 0, kDebugTri = 1, kDebugInst = 2, kDebugQueue = 3, kDebugList = 4, kDebugStack = 5,
                   kDebugSlots = 8 };

// Aperture polygons with at most kPolyMaxSides sides read their vertex
// directions from DevScene::polygon (k_polygon_table).
constexpr uint32_t kPolyMaxSides = 30, kPolyStride = kPolyMaxSides + 2;

// Reference subframe byte offsets (scene.hh:26-34, verified in include/ptg.h users)
enum : uint32_t {
    SF_STRIDE = 160,
    SF_TLAS = 0,                  // bvh {node_count, node_offset}
    SF_CAM = 16,                  // camera: orientation rows @0,16,32; position @48; aspect @64,
                                  //   inv_focal @68, focal_dist @72, ap_angle @76, ap_polygon @80, ap_radius @84
    SF_LIGHT = 112,               // light: direction @0, color @16, cos_solid_angle @32
};

} // namespace ptg
