// Host closest-hit query with the reference ray_query semantics
// (ray_query.hh:111-290).  Only the host scene construction uses it
// (terrain_trace, scene.cc:93-133); rendering runs on the GPU.
#include "scene_internal.h"
#include "hmath.h"

namespace ptg {
namespace {

using namespace hm;

struct Level {                 // ray_query_context (ray_query.hh:40-61)
    ptg_bvh as;
    f3 origin, dir, inv_dir;   // dir holds S (shear constants) for a BLAS level
    uint32_t link_offset = 0, node = 0;
};

float safe_rcp(float d) { return d == 0 ? (float)1e40 : 1.0f / d; }   // 1/dir, 0 -> 1e40 (= +inf)

uint32_t octant(f3 d) { return (d.x > 0 ? 1u : 0u) | (d.y > 0 ? 2u : 0u) | (d.z > 0 ? 4u : 0u); }

// ray_query_traverse (ray_query.hh:184-223)
uint32_t walk(Level& L, const ptg_bvh_node* nodes, const ptg_bvh_link* links, float tmin, float tmax)
{
    while(L.node < L.as.node_count)
    {
        const ptg_bvh_node& n = nodes[L.as.node_offset + L.node];
        const ptg_bvh_link& k = links[L.link_offset + L.node];
        f3 t0 = (v3(n.min_x, n.min_y, n.min_z) - L.origin) * L.inv_dir;
        f3 t1 = (v3(n.max_x, n.max_y, n.max_z) - L.origin) * L.inv_dir;
        f3 lo = vmin(t0, t1), hi = vmax(t0, t1);
        float near_ = fmaxf_(lo.x, fmaxf_(lo.y, lo.z));
        float far_ = fminf_(hi.x, fminf_(hi.y, hi.z));
        if(near_ <= far_ && far_ > tmin && near_ < tmax)
        {
            uint32_t a = k.accept & 0x7FFFFFFFu;
            if(a != k.accept) { L.node = k.cancel; return a; }
            L.node = a;
        }
        else L.node = k.cancel;
    }
    return 0xFFFFFFFFu;
}

} // namespace

HostHit host_closest_hit(const ptg_bvh& tlas, const ptg_tlas_instance* instances, const ptg_bvh_node* nodes,
                         const ptg_bvh_link* links, const uint32_t* indices, const ptg_float3* pos,
                         ptg_float3 origin, ptg_float3 dir, float tmin, float tmax)
{
    Level top, bot;
    top.as = tlas;
    top.origin = origin;
    top.dir = dir;
    top.inv_dir = v3(safe_rcp(dir.x), safe_rcp(dir.y), safe_rcp(dir.z));
    top.link_offset = tlas.node_offset * 8 + octant(dir) * tlas.node_count;
    int axis = -1;                           // blas_axis: -1 while in the TLAS
    ptg_mesh mesh{};
    HostHit best{v3(0, 0, 0), -1.0f, 0xFFFFFFFFu, 0, false};
    HostHit cand = best;
    for(;;)
    {
        uint32_t leaf = walk(axis < 0 ? top : bot, nodes, links, tmin, tmax);
        if(leaf == 0xFFFFFFFFu)
        {
            if(axis < 0) break;
            axis = -1;
            continue;
        }
        if(axis < 0)
        {   // ray_query_enter_blas (ray_query.hh:153-182)
            cand.instance_id = leaf;
            const ptg_tlas_instance& in = instances[leaf];
            bot.as = in.blas;
            f4 o = mul_m4v4(in.inv_transform, v4(origin.x, origin.y, origin.z, 1));
            bot.origin = v3(o.x, o.y, o.z);
            f3 d = mul_m3v3(extract(in.inv_transform), dir);
            bot.inv_dir = v3(safe_rcp(d.x), safe_rcp(d.y), safe_rcp(d.z));
            bot.link_offset = in.blas.node_offset * 8 + octant(d) * in.blas.node_count;
            bot.node = 0;
            mesh = in.m;
            // ray_triangle_intersection_preprocess (math.hh:340-356)
            f3 ad = v3((float)std::fabs(d.x), (float)std::fabs(d.y), (float)std::fabs(d.z));
            f3 rd = d;
            axis = 2;
            if(ad.x > ad.y && ad.x > ad.z) { axis = 0; rd = v3(d.z, d.y, d.x); }
            else if(ad.y > ad.z) { axis = 1; rd = v3(d.x, d.z, d.y); }
            bot.dir = v3(rd.x, rd.y, 1.0f) * (1.0f / rd.z);
            continue;
        }
        // ray_query_test_triangle + ray_triangle_intersection (ray_query.hh:225-246, math.hh:358-401)
        cand.primitive_id = leaf;
        const uint32_t* tri = indices + mesh.index_offset + size_t(leaf) * 3;
        f3 A = pos[mesh.base_vertex_offset + tri[0]] - bot.origin;
        f3 B = pos[mesh.base_vertex_offset + tri[1]] - bot.origin;
        f3 C = pos[mesh.base_vertex_offset + tri[2]] - bot.origin;
        f3 x = v3(A.x, B.x, C.x), y = v3(A.y, B.y, C.y), z = v3(A.z, B.z, C.z);
        if(axis == 0) { x = z; z = v3(A.x, B.x, C.x); }
        else if(axis == 1) { y = z; z = v3(A.y, B.y, C.y); }
        const f3 S = bot.dir;
        x = x - S.x * z;
        y = y - S.y * z;
        f3 uvw = cross(y, x);
        float det = uvw.x + uvw.y + uvw.z;
        f3 uvt = v3(uvw.x, uvw.y, dot(uvw, S.z * z)) * (1.0f / det);
        bool back = det < 0;
        if(S.z < 0) back = !back;
        if(axis != 2) back = !back;
        bool hit = det != 0.0f && uvt.z >= 0.0f &&
                   ((uvw.x >= 0.0f && uvw.y >= 0.0f && uvw.z >= 0.0f) ||
                    (uvw.x <= 0.0f && uvw.y <= 0.0f && uvw.z <= 0.0f));
        cand.thit = uvt.z;
        cand.bary = v3(uvt.x, uvt.y, 1.0f - uvt.x - uvt.y);
        cand.back_face = back;
        if(hit && cand.thit < tmax && cand.thit > tmin)
        {   // ray_query_confirm (ray_query.hh:280-290)
            best = cand;
            tmax = cand.thit;
        }
    }
    return best;
}

} // namespace ptg
