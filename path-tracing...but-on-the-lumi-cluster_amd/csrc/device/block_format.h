// Block BVH records: the walk's traversal data, shared by the host packer
// (host/block_bvh.cpp) and the device walker (BlockWalker, device/path_tracer.h).
//
// The reference stores a BVH as nodes (bvh.hh:45-51, 24 B AABB) plus eight
// stackless link orders (bvh.hh:53-67), one per ray-direction octant, and
// walks it node by node along `accept` / `cancel`: one dependent 32 B gather
// per node visit (ray_query.hh:184-223).  The links encode one fixed order:
// the children of an inner node in build (BFS) order, reversed exactly when
// the ray's direction is not positive on the node's split axis
// (bvh.cc:173-191).  Every leaf the walk reaches is therefore met in one
// depth-first order per octant, and a leaf is reached iff its own box test
// and those of all its ancestors pass, each at its own time (tmax shrinks as
// hits are confirmed).
//
// Two facts let a walk test far fewer boxes with the same outcome:
//  1. Containment.  Every box contains its children's boxes (each is the
//     fmin/fmax union of the leaf boxes below it, bvh.cc:65-80, 198-201; the
//     packer checks it), and the slab test
//     `near <= far && far > tmin && near < tmax` (ray_query.hh:197-207) is
//     monotone under box inclusion in IEEE arithmetic (subtraction and
//     multiplication by the same reciprocal are monotone; an infinite
//     reciprocal yields a NaN only on a slab plane, where the child fails
//     too).  So a child that passes at some tmax has a parent that passes at
//     any tmax at least as large - in particular at the parent's own, earlier
//     test.  Skipping inner box tests never changes which leaves are reached.
//  2. Deferred tests.  `near` and `far` do not depend on tmax, and tmax only
//     shrinks.  A box tested early with a larger tmax, rejected, is rejected
//     by the reference too; accepted, it is re-checked with `near < tmax` at
//     the time the reference would test it.
// Leaf boxes gate the triangle tests and BLAS entries, so they are always
// decided at their own time (fact 2); inner boxes are tested only to prune.
//
// Layout.  The binary SAH tree (with multi-leaf buckets, split into groups
// of at most four) is collapsed into 4-wide blocks: a block holds up to four
// descendants of one node (its children, some replaced by their own
// children).  Each block is stored once per ray octant (8 x 4 entries): in
// octant o's copy the entries are in the order a ray of that octant meets
// them, and each box is stored as (near planes, far planes) for that
// octant's direction signs, so with finite reciprocals the slab test needs no
// per-axis min/max (t of the near plane is the reference's fmin(t0, t1) of
// that axis, the far plane's its fmax).  A walk step loads one copy (112 B
// used of 128, seven 16-byte loads with no dependency between them), tests all four
// boxes, continues with the first passing entry and pushes the others, each
// with its `near`, onto a per-lane stack in reverse order; a popped entry is
// re-checked with `near < tmax` (fact 2).  Leaves are thus met in the
// reference's order with the reference's tmax: identical hits, ties and
// back-face flags.
//
//   BlockCopy (128 B: seven 16-byte rows used)
//     rows 0-3   entry j: near.xyz | a
//     rows 4-6   the four entries' far.xyz, packed (f[3j .. 3j+2])
//     a: kBeLeaf | payload   leaf (BLAS: triangle index in the mesh,
//                            TLAS: instance index), payload < 2^28
//        kBeNone             unused slot (planes at +-inf: near +inf, far -inf for the copy's octant; never passes)
//        otherwise           block index of the child's own block
//   octant o's copy of block k: blocks[k * 8 + o]
// A BVH's handle is its root block's index; the root's own box is never
// tested (fact 1).  The records are ~113 MB for the BLASes the animation
// uses, against 8 x 581k x 64 B = 298 MB of per-octant paired node records.
#pragma once
#include <stdint.h>

namespace ptg {

#ifndef PTG_BLOCK_WIDTH
#define PTG_BLOCK_WIDTH 4   // other widths only in the CPU model (tools/walk_sim, WIDTH=8)
#endif
constexpr uint32_t kBlockWidth = PTG_BLOCK_WIDTH;
constexpr uint32_t kBlockCopies = 8;   // a block: one copy per octant

struct alignas(16) BlockCopy {
    struct Near {
        float x, y, z;
        uint32_t a;
    } n[kBlockWidth];                  // rows 0-3
    float f[3 * kBlockWidth];          // rows 4-6: entry j's far planes at f[3j .. 3j+2]
    uint32_t pad[(128 - (28 * kBlockWidth) % 128) % 128 / 4];   // row 7 (keeps copies on 128-byte lines)
};
static_assert(sizeof(BlockCopy) % 128 == 0 && (kBlockWidth != 4 || sizeof(BlockCopy) == 128),
              "BlockCopy is one 128-byte line");

constexpr uint32_t kBeLeaf = 0x80000000u;
constexpr uint32_t kBeNone = 0x40000000u;
constexpr uint32_t kBeIndex = 0x0FFFFFFFu;   // 28-bit block indices and payloads
// The walker's stack words are entry words (a block index, or kBeLeaf |
// payload); a leaf word sits on top of its `near` (float bits).  kBePop
// (a leaf word no payload can produce) means "take the next stack entry".
constexpr uint32_t kBePop = 0xFFFFFFFFu;
// A parked triangle that is an any-hit walk's occluder candidate
// (BlockWalker::try_candidate): its leaf box is tested from its vertices.
constexpr uint32_t kBeCand = 0x20000000u;

} // namespace ptg
