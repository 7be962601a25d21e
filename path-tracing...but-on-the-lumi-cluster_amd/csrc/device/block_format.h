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
// children).  Each block is stored ONCE (one 128-byte line), its entries in
// the canonical order - the order of a ray whose direction is positive on
// every axis (octant 7: no child list reversed) - and its boxes as planes
// in struct-of-arrays rows:
//
//   BlockCopy (128 B: seven 16-byte rows used)
//     row 2a     the four entries' min planes on axis a (a = x, y, z)
//     row 2a + 1 the four entries' max planes on axis a
//     row 6      the four entry words a[j]
//   a: kBeLeaf | payload   leaf (BLAS: triangle index in the mesh,
//                          TLAS: instance index), payload < 2^24
//      kBeNone             unused slot (box empty: min +inf, max -inf; never passes)
//      otherwise           block index of the child's own block (< 2^24)
//   bits 24-27 of a[0] and bits 24-26 of a[1]: the block's order id (below)
//
// A ray reads its near planes from the row its direction's sign names (min
// for a positive component, else max) and its far planes from the other:
// the row offsets are per lane, so the load addresses do the selection and
// the slab test needs no per-axis min/max (BlockWalker::node_block).
//
// The entry order for octant o is the reference's: depth-first through the
// block's expanded nodes, each one's children forward or reversed by the
// sign of its axis (bvh.cc:177-181).  It depends only on the block's shape
// and its expanded nodes' axes, so the 8 orders of a block are one of the
// kOrderTables order tables (host/block_bvh.cpp enumerates them: every tree
// of at most four entries, every axis choice); the block names its table
// by id.  Table byte o: bits 2p..2p+1 = the canonical index of the entry a
// ray of octant o meets p-th.
//
// The records are ~14 MB for the BLASes the animation uses (one line per
// block; against 113 MB with a copy per octant, round 5, whose incoherent
// bounce rays touched up to eight lines per block: tools/walk_sim COPIES).
// A handle (TLAS root, BLAS root) is its root block's index; the root's own
// box is never tested (fact 1).
#pragma once
#include <stdint.h>

namespace ptg {

constexpr uint32_t kBlockWidth = 4;   // (8-wide blocks were modelled and measured slower, DESIGN.md 4.2;
                                      //  the order tables' 2-bit entry fields assume 4)
constexpr uint32_t kBlockCopies = 1;   // a block: one line (entries in canonical order + an order id)

struct alignas(16) BlockCopy {
    float p[6][kBlockWidth];           // rows 0-5: plane[2 * axis + (0 min | 1 max)][entry]
    uint32_t a[kBlockWidth];           // row 6: entry words (+ order id bits in a[0], a[1])
    uint32_t pad[(128 - (28 * kBlockWidth) % 128) % 128 / 4];   // row 7 (keeps blocks on 128-byte lines)
};
static_assert(sizeof(BlockCopy) % 128 == 0 && (kBlockWidth != 4 || sizeof(BlockCopy) == 128),
              "BlockCopy is one 128-byte line");

constexpr uint32_t kBeLeaf = 0x80000000u;
constexpr uint32_t kBeNone = 0x40000000u;
constexpr uint32_t kBeIndex = 0x00FFFFFFu;   // 24-bit block indices and payloads
constexpr uint32_t kBeOrderShift = 24;       // order id: a[0] bits 24-27 (low 4 bits), a[1] bits 24-26 (high 3)
constexpr uint32_t kOrderTables = 112;       // distinct order tables of <= 4-entry blocks (host/block_bvh.cpp)
static_assert(kOrderTables <= 128, "order ids take 7 bits");
// The walker's stack words are entry words (a block index, or kBeLeaf |
// payload, possibly with order-id bits above the index: masked with kBeIndex
// wherever an index is taken); a leaf word sits on top of its `near` (float
// bits).  kBePop (a leaf word no payload can produce) means "take the next
// stack entry".
constexpr uint32_t kBePop = 0xFFFFFFFFu;
// A parked triangle that is an any-hit walk's occluder candidate
// (BlockWalker::try_candidate): its leaf box is tested from its vertices.
constexpr uint32_t kBeCand = 0x20000000u;

// The order id a block's words carry.
inline constexpr uint32_t block_order_id(uint32_t a0, uint32_t a1)
{
    return ((a0 >> kBeOrderShift) & 15u) | (((a1 >> kBeOrderShift) & 7u) << 4);
}
// canonical index of the entry a ray of octant o meets at position p, from
// its table byte
inline constexpr uint32_t order_entry(uint32_t table_byte, uint32_t p) { return (table_byte >> (2u * p)) & 3u; }

} // namespace ptg
