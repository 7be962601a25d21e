// Internal C++ interface of the host-side scene restatement.
#pragma once
#include "ptg.h"
#include <string>
#include <unordered_map>
#include <utility>
#include <vector>

namespace ptg {

// mesh_buffers (mesh.hh:32-44)
struct MeshBuffers {
    std::vector<uint32_t> indices;
    std::vector<ptg_float3> pos;
    std::vector<ptg_float3> normal;
    std::vector<ptg_float4> albedo;
    std::vector<ptg_float4> material;
};

// bvh_buffers (bvh.hh:88-92)
struct BvhBuffers {
    std::vector<ptg_bvh_node> nodes;
    std::vector<ptg_bvh_link> links;
};

// load_mesh (mesh.cc:110-265).  Throws std::runtime_error on I/O failure.
ptg_mesh load_obj_mesh(MeshBuffers& mb, const std::string& obj_path);

// One BVH leaf candidate: bounds + payload (bvh.cc:11-16).
struct BuildLeaf {
    ptg_float3 min, max;
    uint32_t index;
};

// build_generic_bvh (bvh.cc:195-229): appends nodes + 8 link orders.
ptg_bvh build_bvh(std::vector<BuildLeaf>& leaves, BvhBuffers& out, float traversal_cost = 2.0f);
#ifdef PTG_MODEL_HOOKS
extern float g_model_blas_traversal_cost;   // tools/walk_sim ANYHIER: the BLAS builds' SAH traversal cost
#endif
// build_blas (bvh.cc:231-250)
ptg_bvh build_blas(const ptg_mesh& m, const MeshBuffers& mb, BvhBuffers& out);
// build_tlas (bvh.cc:252-284): instances[i] with leaf payload ids[i]
ptg_bvh build_tlas(size_t count, const ptg_tlas_instance* const* instances, const uint32_t* ids,
                   const BvhBuffers& in, BvhBuffers& out);
// pop_bvh (bvh.cc:286-292)
void pop_bvh(BvhBuffers& bc, ptg_bvh& as);

// Host closest-hit query (ray_query.hh semantics) - used by load_scene's
// object placement (scene.cc:93-133).
struct HostHit {
    ptg_float3 bary;
    float thit;
    uint32_t instance_id, primitive_id;
    bool back_face;
};
HostHit host_closest_hit(const ptg_bvh& tlas, const ptg_tlas_instance* instances, const ptg_bvh_node* nodes,
                         const ptg_bvh_link* links, const uint32_t* indices, const ptg_float3* pos,
                         ptg_float3 origin, ptg_float3 dir, float tmin, float tmax);

} // namespace ptg

// struct scene (scene.hh:40-65)
struct ptg_scene {
    ptg::MeshBuffers mesh_buf;
    ptg::BvhBuffers bvh_buf;
    std::unordered_map<std::string, std::pair<ptg_mesh, ptg_bvh>> meshes;
    std::vector<ptg_tlas_instance> instances;
    uint32_t static_instance_count = 0;
    size_t static_node_count = 0;
    std::vector<ptg_subframe> subframes;
    ptg_render_config cfg;
};

namespace ptg {
void set_last_error(const std::string& msg);
// Host worker threads one of this process's pools may use: the CPUs this
// process may run on (affinity mask, cgroup CPU quota) shared by the ranks of
// one node (LOCAL_WORLD_SIZE, set by torch.distributed.run), at least 1;
// ptg_set_host_threads overrides it.
unsigned host_threads();
}
