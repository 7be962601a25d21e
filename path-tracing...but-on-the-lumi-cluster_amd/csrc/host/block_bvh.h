// Host packer of the block BVH records (device/block_format.h).
#pragma once
#include "ptg.h"
#include "../device/block_format.h"
#include <string>
#include <vector>

namespace ptg {

unsigned host_threads();   // scene.cpp: this process's share of the host's CPUs

struct BlockBvh {
    uint32_t root = 0;          // root block index (absolute: block_base + position)
    uint32_t blocks = 0;        // blocks appended
    uint32_t stack_entries = 0; // most stack entries a walk of this BVH can hold
    uint32_t max_payload = 0;   // largest leaf payload
};

// Packs one BVH given in the reference layout - nodes[0..count) and the eight
// link orders links[o * count + i] (bvh.cc:195-229) - appending its blocks
// (kBlockCopies copies each, one per octant) to `out`.  Child block
// indices are block_base + position in `out` / kBlockCopies.  Checked, with an error in `err`:
//   - the links are the reference builder's: a tree rooted at node 0 whose
//     every order lists each node's children forward, or reversed when the
//     octant's sign on the node's axis is not positive (bvh.cc:173-191);
//   - every box contains its children's boxes (the walk skips inner boxes);
//   - leaf payloads are below payload_limit (and 2^28).
bool pack_block_bvh(const ptg_bvh_node* nodes, const ptg_bvh_link* links, uint32_t count, uint32_t block_base,
                    uint32_t payload_limit, std::vector<BlockCopy>& out, BlockBvh& info, std::string& err);

} // namespace ptg

#include <unordered_map>

namespace ptg {

// Whether every leaf box of a BLAS (nodes[0..count), links in the reference
// layout) is exactly the bounds of its triangle's three positions as the
// reference's builder computes them (bvh.cc:243-246: fmin / fmax, the float
// overloads, whose tie rule fixes the sign of zero bounds) - the any-hit
// walk tests a candidate triangle's leaf box from its vertices
// (BlockWalker::try_candidate).  `indices` and `pos` are the scene's arrays;
// the mesh is (index_offset, triangle_count, base_vertex_offset).  Built by
// the host compiler with the builder's flags (host/hmath.h), so the
// comparison is bit for bit: hipcc's std::fmin (llvm.minnum) may pick either
// zero of a +0 / -0 tie.
bool leaf_boxes_are_vertex_bounds(const ptg_bvh_node* nodes, const ptg_bvh_link* links, uint32_t count,
                                  const uint32_t* indices, size_t index_count, const ptg_float3* pos, size_t vertex_count,
                                  uint32_t index_offset, uint32_t triangle_count, uint32_t base_vertex_offset);

// A packed BLAS in the block cache.
struct BlasRecord {
    uint32_t root = 0;          // root block
    uint32_t count = 0;         // node count it was packed with
    uint32_t max_payload = 0;   // largest triangle index its leaves name
};

// What one frame upload adds to the block buffer [BLAS blocks][TLAS blocks].
struct FramePack {
    uint32_t blas_base = 0;                 // block index of new_blas[0]
    uint32_t tlas_base = 0;                 // block index of tlas[0]
    std::vector<BlockCopy> new_blas;       // BLASes no earlier frame packed
    std::vector<BlockCopy> tlas;           // this frame's TLASes, one per subframe
    std::unordered_map<uint32_t, BlasRecord> new_records;
    std::vector<uint32_t> tlas_root;        // per subframe
    std::vector<uint32_t> inst_root;        // per instance: its BLAS's root block
    uint32_t blas_stack = 0, tlas_stack = 0;
    uint32_t total_blocks() const { return tlas_base + uint32_t(tlas.size() / kBlockCopies); }
    uint32_t stack_bound() const { return blas_stack + tlas_stack; }   // stack entries a walk can hold
};

// The BLAS blocks packed so far and the packing of a frame's handles: the
// host half of ptg_upload_frame, kept free of device code so the CPU tests
// (tools/walk_sim.cpp) run exactly what the upload runs.
struct BlockCache {
    std::vector<BlockCopy> blas;                         // committed BLAS blocks
    std::unordered_map<uint32_t, BlasRecord> records;     // BLAS node_offset -> record
    uint32_t blas_stack = 0;                              // largest committed BLAS stack bound

    void clear()
    {
        blas.clear();
        records.clear();
        blas_stack = 0;
    }
    // Checks every handle of the frame (BLAS and mesh ranges, TLAS ranges,
    // leaf payloads, block links) and packs the BLASes not yet cached plus
    // every subframe's TLAS.  `static_nodes/links` are the scene's BLAS
    // arrays (reference layout), `frame_nodes/links` the frame's TLAS arrays
    // starting at global node `first_node`.  Returns PTG_OK, or PTG_E_RANGE
    // with the reason in `err`; the cache is not modified.
    int pack_frame(const ptg_bvh_node* static_nodes, const ptg_bvh_link* static_links, size_t static_count,
                   size_t index_count, size_t vertex_count, const ptg_subframe* subframes, size_t subframe_count,
                   const ptg_tlas_instance* instances, size_t instance_count, const ptg_bvh_node* frame_nodes,
                   const ptg_bvh_link* frame_links, size_t first_node, size_t frame_node_count, FramePack& fp,
                   std::string& err) const;
    // Adds a successfully uploaded frame's new BLASes to the cache.
    void commit(FramePack& fp);
};

} // namespace ptg
