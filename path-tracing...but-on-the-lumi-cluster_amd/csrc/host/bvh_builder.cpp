// BVH construction - restatement of bvh.cc (build_recursive_sah :43-143,
// BFS numbering :145-168, stackless link orders :170-193).
//
// The node order and the eight link orders define the traversal order of the
// hot path, and ties between equal hit distances are resolved by that order
// (ray_query.hh:245), so the output must match the reference exactly:
//   * full-sweep SAH over the three axes, leaves sorted by centroid
//     (max + min) with the leaf index as tie-break - a strict total order, so
//     the sorted sequence is unique whatever sort algorithm produces it;
//   * cost = (i+1)*area(left) + (n-1-i)*area(right), half-surface areas
//     xy + zx + yz, normalised by the parent's area plus a traversal cost of 2;
//     when n <= that cost the node keeps all its leaves as children;
//   * nodes numbered breadth first; for each of the 8 ray-direction octants a
//     link array {accept, cancel} whose child order follows the sign of the
//     node's split axis.
#include "scene_internal.h"
#include "hmath.h"
#include <algorithm>
#include <cfloat>

namespace ptg {
#ifdef PTG_MODEL_HOOKS
float g_model_blas_traversal_cost = 2.0f;
#endif
namespace {

using namespace hm;

struct TreeNode {
    f3 min, max;
    int axis = -1;
    uint32_t payload = 0;            // leaf: primitive / instance id
    uint32_t number = 0;             // BFS index
    std::vector<uint32_t> kids;      // indices into the node pool; empty = leaf
};

struct Builder {
    float traversal_cost = 2.0f;     // bvh.cc:111-112
    std::vector<TreeNode> pool;
    std::vector<f3> pre_min, pre_max, suf_min, suf_max;

    static float half_area(f3 s) { return s.x * s.y + s.z * s.x + s.y * s.z; }

    static void sort_by_axis(BuildLeaf* b, BuildLeaf* e, int axis)
    {
        std::sort(b, e, [axis](const BuildLeaf& p, const BuildLeaf& q) {
            float cp = comp(p.max, axis) + comp(p.min, axis);
            float cq = comp(q.max, axis) + comp(q.min, axis);
            if(cp < cq) return true;
            if(cp > cq) return false;
            return p.index < q.index;
        });
    }

    // build_recursive_sah, bvh.cc:43-143.  `self` bounds are set by the caller.
    void split(BuildLeaf* leaves, uint32_t n, uint32_t self)
    {
        pool[self].axis = -1;
        if(n == 1)
        {
            pool[self].payload = leaves[0].index;
            return;
        }
        float best = FLT_MAX;
        uint32_t best_split = 0;
        f3 bmin0{}, bmax0{}, bmin1{}, bmax1{};
        pre_min.resize(n); pre_max.resize(n); suf_min.resize(n); suf_max.resize(n);
        for(int axis = 0; axis < 3; ++axis)
        {
            sort_by_axis(leaves, leaves + n, axis);
            // prefix bounds of leaves[0..i] and suffix bounds of leaves[i+1..n-1],
            // accumulated in the reference's order (fmin(accumulated, new leaf))
            for(uint32_t i = 0; i + 1 < n; ++i)
            {
                pre_min[i] = i == 0 ? leaves[0].min : vmin(pre_min[i - 1], leaves[i].min);
                pre_max[i] = i == 0 ? leaves[0].max : vmax(pre_max[i - 1], leaves[i].max);
                uint32_t k = n - 1 - i;
                suf_min[k - 1] = i == 0 ? leaves[k].min : vmin(suf_min[k], leaves[k].min);
                suf_max[k - 1] = i == 0 ? leaves[k].max : vmax(suf_max[k], leaves[k].max);
            }
            for(uint32_t i = 0; i + 1 < n; ++i)
            {
                float a0 = half_area(pre_max[i] - pre_min[i]);
                float a1 = half_area(suf_max[i] - suf_min[i]);
                float cost = float(i + 1) * a0 + float(n - 1 - i) * a1;
                if(cost < best)
                {
                    bmin0 = pre_min[i]; bmax0 = pre_max[i];
                    bmin1 = suf_min[i]; bmax1 = suf_max[i];
                    best = cost;
                    best_split = i + 1;
                    pool[self].axis = axis;
                }
            }
        }
        f3 size = pool[self].max - pool[self].min;
        best /= half_area(size);
        best += traversal_cost;
        const bool keep_leaves = float(n) <= best;
        if(keep_leaves)
        {
            int ax = 2;
            if(size.x > size.y && size.x > size.z) ax = 0;
            else if(size.y > size.z) ax = 1;
            pool[self].axis = ax;
        }
        sort_by_axis(leaves, leaves + n, pool[self].axis);
        if(keep_leaves)
        {
            for(uint32_t i = 0; i < n; ++i)
            {
                TreeNode leaf;
                leaf.min = leaves[i].min;
                leaf.max = leaves[i].max;
                leaf.payload = leaves[i].index;
                pool.push_back(leaf);
                pool[self].kids.push_back(uint32_t(pool.size() - 1));
            }
            return;
        }
        TreeNode c0, c1;
        c0.min = bmin0; c0.max = bmax0;
        c1.min = bmin1; c1.max = bmax1;
        pool.push_back(c0);
        uint32_t i0 = uint32_t(pool.size() - 1);
        pool.push_back(c1);
        uint32_t i1 = uint32_t(pool.size() - 1);
        pool[self].kids = {i0, i1};
        split(leaves, best_split, i0);
        split(leaves + best_split, n - best_split, i1);
    }

    // save_traversal_links (bvh.cc:170-193) for one octant
    void links(const bool sign[3], uint32_t node, uint32_t cancel, ptg_bvh_link* out) const
    {
        const TreeNode& t = pool[node];
        if(t.kids.empty())
        {
            out[t.number] = ptg_bvh_link{0x80000000u | t.payload, cancel};
            return;
        }
        const bool reverse = !sign[t.axis];
        const size_t m = t.kids.size();
        for(size_t i = 0; i < m; ++i)
        {
            uint32_t child = t.kids[reverse ? m - 1 - i : i];
            if(i == 0) out[t.number] = ptg_bvh_link{pool[child].number, cancel};
            uint32_t next = cancel;
            if(i + 1 < m) next = pool[t.kids[reverse ? m - 2 - i : i + 1]].number;
            links(sign, child, next, out);
        }
    }
};

} // namespace

ptg_bvh build_bvh(std::vector<BuildLeaf>& leaves, BvhBuffers& bc, float traversal_cost)
{
    Builder b;
    b.traversal_cost = traversal_cost;
    b.pool.reserve(leaves.size() * 2 + 1);
    TreeNode root;
    root.min = v3(FLT_MAX, FLT_MAX, FLT_MAX);
    root.max = v3(-FLT_MAX, -FLT_MAX, -FLT_MAX);
    for(const BuildLeaf& l: leaves)
    {
        root.min = vmin(root.min, l.min);
        root.max = vmax(root.max, l.max);
    }
    b.pool.push_back(root);
    b.split(leaves.data(), uint32_t(leaves.size()), 0);

    ptg_bvh out;
    out.node_offset = uint32_t(bc.nodes.size());
    // breadth-first numbering and node emission (bvh.cc:145-168)
    std::vector<uint32_t> layer{0}, next;
    uint32_t counter = 0;
    while(!layer.empty())
    {
        for(uint32_t id: layer)
        {
            TreeNode& t = b.pool[id];
            bc.nodes.push_back(ptg_bvh_node{t.min.x, t.min.y, t.min.z, t.max.x, t.max.y, t.max.z});
            t.number = counter++;
            for(uint32_t k: t.kids) next.push_back(k);
        }
        layer.swap(next);
        next.clear();
    }
    out.node_count = uint32_t(bc.nodes.size()) - out.node_offset;
    bc.links.resize(bc.links.size() + size_t(8) * out.node_count);
    for(int o = 0; o < 8; ++o)
    {
        const bool sign[3] = {bool(o & 1), bool(o & 2), bool(o & 4)};
        b.links(sign, 0, 0xFFFFFFFFu, bc.links.data() + size_t(8) * out.node_offset + size_t(o) * out.node_count);
    }
    return out;
}

ptg_bvh build_blas(const ptg_mesh& m, const MeshBuffers& mb, BvhBuffers& out)
{
    std::vector<BuildLeaf> leaves;
    leaves.reserve(m.triangle_count);
    for(uint32_t i = 0; i < m.triangle_count; ++i)
    {
        const uint32_t* tri = &mb.indices[m.index_offset + size_t(i) * 3];
        f3 p0 = mb.pos[m.base_vertex_offset + tri[0]];
        f3 p1 = mb.pos[m.base_vertex_offset + tri[1]];
        f3 p2 = mb.pos[m.base_vertex_offset + tri[2]];
        leaves.push_back(BuildLeaf{vmin(p0, vmin(p1, p2)), vmax(p0, vmax(p1, p2)), i});
    }
#ifdef PTG_MODEL_HOOKS
    // tools/walk_sim ANYHIER (model builds only): BLASes with another SAH
    // traversal cost, the same leaves and leaf boxes
    return build_bvh(leaves, out, g_model_blas_traversal_cost);
#else
    return build_bvh(leaves, out);
#endif
}

ptg_bvh build_tlas(size_t count, const ptg_tlas_instance* const* instances, const uint32_t* ids,
                   const BvhBuffers& in, BvhBuffers& out)
{
    std::vector<BuildLeaf> leaves;
    leaves.reserve(count);
    for(size_t i = 0; i < count; ++i)
    {
        const ptg_tlas_instance& inst = *instances[i];
        const ptg_bvh_node& root = in.nodes[inst.blas.node_offset];
        const f3 lo = v3(root.min_x, root.min_y, root.min_z), hi = v3(root.max_x, root.max_y, root.max_z);
        BuildLeaf leaf;
        leaf.index = ids[i];
        // the 8 corners of the BLAS root box, as enumerated in bvh.cc:270-280
        for(int a = 0; a < 8; ++a)
        {
            f4 corner = v4((a & 1) ? hi.x : lo.x, (a & 2) ? lo.y : hi.y, (a & 4) ? lo.z : hi.z, 1);
            f4 w = mul_m4v4(inst.transform, corner);
            f3 c = v3(w.x, w.y, w.z);
            leaf.min = a == 0 ? c : vmin(c, leaf.min);
            leaf.max = a == 0 ? c : vmax(c, leaf.max);
        }
        leaves.push_back(leaf);
    }
    return build_bvh(leaves, out);
}

void pop_bvh(BvhBuffers& bc, ptg_bvh& as)
{
    if(as.node_count == 0) return;
    bc.nodes.resize(as.node_offset);
    bc.links.resize(size_t(as.node_offset) * 8u);
    as.node_count = 0;
}

} // namespace ptg
