// Block BVH packer (device/block_format.h): the reference's nodes and eight
// link orders (bvh.cc:145-229) -> 4-wide blocks, breadth-first, so the top
// levels every ray walks share cache lines.
#include "block_bvh.h"
#include "hmath.h"
#include <algorithm>
#include <cstring>
#include <thread>
#include <unordered_map>
#include <cmath>
#include <limits>

namespace ptg {

namespace {

struct Tree {
    std::vector<std::vector<uint32_t>> kids;   // children in build (forward) order
    std::vector<uint32_t> axis;                // split / sort axis (orders the children)
    std::vector<uint32_t> payload;             // leaves: kBeLeaf | payload, else 0
    std::vector<ptg_bvh_node> box;
    bool leaf(uint32_t n) const { return (payload[n] & kBeLeaf) != 0; }
};

bool contains(const ptg_bvh_node& p, const ptg_bvh_node& c)
{
    return p.min_x <= c.min_x && p.min_y <= c.min_y && p.min_z <= c.min_z && c.max_x <= p.max_x && c.max_y <= p.max_y &&
           c.max_z <= p.max_z;
}

double area(const ptg_bvh_node& b)
{
    const double x = double(b.max_x) - b.min_x, y = double(b.max_y) - b.min_y, z = double(b.max_z) - b.min_z;
    return x * y + y * z + z * x;
}

// The tree behind the links, checked against the reference builder's rules.
bool derive(const ptg_bvh_node* nodes, const ptg_bvh_link* links, uint32_t count, uint32_t payload_limit, Tree& t,
            std::string& err)
{
    auto L = [&](uint32_t o, uint32_t i) -> const ptg_bvh_link& { return links[size_t(o) * count + i]; };
    t.kids.assign(count, {});
    t.axis.assign(count, 0);
    t.payload.assign(count, 0);
    t.box.assign(nodes, nodes + count);
    std::vector<uint8_t> parents(count, 0);
    for(uint32_t n = 0; n < count; ++n)
    {
        const ptg_bvh_link& l7 = L(7, n);   // order 7: every sign positive, nothing reversed (bvh.cc:178)
        if(l7.accept & 0x80000000u)
        {
            const uint32_t p = l7.accept & 0x7FFFFFFFu;
            if(p >= payload_limit || p > kBeIndex)
            {
                err = "leaf payload " + std::to_string(p) + " out of range (limit " + std::to_string(payload_limit) + ")";
                return false;
            }
            for(uint32_t o = 0; o < 8; ++o)
                if(L(o, n).accept != l7.accept) { err = "leaf payload differs between link orders"; return false; }
            t.payload[n] = kBeLeaf | p;
            continue;
        }
        uint32_t c = l7.accept;
        t.kids[n].reserve(2);
        for(;;)
        {
            if(c >= count || c == 0) { err = "link outside the BVH"; return false; }
            if(parents[c]++) { err = "node with two parents"; return false; }
            t.kids[n].push_back(c);
            const uint32_t nx = L(7, c).cancel;
            if(nx == l7.cancel) break;
            c = nx;
        }
        const std::vector<uint32_t>& k = t.kids[n];
        bool found = k.size() < 2;   // one child: the order is moot
        for(uint32_t a = 0; a < 3 && !found; ++a)
            if(L(1u << a, n).accept == k[0]) { t.axis[n] = a; found = true; }
        if(!found) { err = "child order matches no axis"; return false; }
        for(uint32_t o = 0; o < 8; ++o)
        {
            const bool rev = ((o >> t.axis[n]) & 1u) == 0;
            auto child = [&](size_t j) { return k[rev ? k.size() - 1 - j : j]; };
            if(L(o, n).accept != child(0)) { err = "accept link is not the first child of its order"; return false; }
            for(size_t j = 0; j < k.size(); ++j)
                if(L(o, child(j)).cancel != (j + 1 < k.size() ? child(j + 1) : L(o, n).cancel))
                { err = "cancel link breaks the child order"; return false; }
        }
        for(uint32_t ch: k)
            if(!contains(t.box[n], t.box[ch])) { err = "box does not contain its child's box"; return false; }
    }
    for(uint32_t n = 1; n < count; ++n)
        if(!parents[n]) { err = "node not reachable from the root"; return false; }
    for(uint32_t o = 0; o < 8; ++o)
        if(L(o, 0).cancel < count) { err = "root has a successor"; return false; }
    return true;
}

// Nodes with more than kBlockWidth children (multi-leaf buckets) get
// consecutive runs of their children grouped under virtual nodes with the
// same axis and the union box: the order rule, and containment, carry over.
void split_wide(Tree& t)
{
    const size_t W = kBlockWidth;
    for(uint32_t n = 0; n < t.kids.size(); ++n)
    {
        while(t.kids[n].size() > W)
        {
            const std::vector<uint32_t> ks = t.kids[n];
            const size_t groups = (ks.size() + W - 1) / W;
            std::vector<uint32_t> out;
            for(size_t i = 0, g = 0; i < ks.size(); ++g)
            {
                const size_t take = std::min(W, (ks.size() - i + (groups - g) - 1) / (groups - g));
                if(take == 1) { out.push_back(ks[i++]); continue; }
                ptg_bvh_node b = t.box[ks[i]];
                for(size_t j = i + 1; j < i + take; ++j)
                {
                    const ptg_bvh_node& c = t.box[ks[j]];
                    b.min_x = std::min(b.min_x, c.min_x); b.min_y = std::min(b.min_y, c.min_y); b.min_z = std::min(b.min_z, c.min_z);
                    b.max_x = std::max(b.max_x, c.max_x); b.max_y = std::max(b.max_y, c.max_y); b.max_z = std::max(b.max_z, c.max_z);
                }
                const uint32_t v = uint32_t(t.kids.size());
                t.kids.emplace_back(ks.begin() + i, ks.begin() + i + take);
                t.axis.push_back(t.axis[n]);
                t.payload.push_back(0);
                t.box.push_back(b);
                out.push_back(v);
                i += take;
            }
            t.kids[n] = out;
        }
    }
}

} // namespace

bool pack_block_bvh(const ptg_bvh_node* nodes, const ptg_bvh_link* links, uint32_t count, uint32_t block_base,
                    uint32_t payload_limit, std::vector<BlockCopy>& out, BlockBvh& info, std::string& err)
{
    if(count == 0) { err = "empty BVH"; return false; }
    Tree t;
    if(!derive(nodes, links, count, payload_limit, t, err)) return false;
    split_wide(t);
    const uint32_t W = kBlockWidth;

    // Block contents: a block root's children, greedily replacing the inner
    // slot with the largest surface area by its own children while they fit.
    struct Blk {
        uint32_t root;
        std::vector<uint32_t> slots, expanded;
    };
    std::vector<Blk> blks;
    std::vector<uint32_t> block_of(t.kids.size(), 0);
    auto make = [&](uint32_t root) {
        Blk b;
        b.root = root;
        b.slots = t.kids[root];
        b.expanded.push_back(root);
        for(;;)
        {
            int best = -1;
            double ba = -1.0;
            for(size_t i = 0; i < b.slots.size(); ++i)
            {
                const uint32_t c = b.slots[i];
                if(t.leaf(c) || b.slots.size() - 1 + t.kids[c].size() > W) continue;
                const double a = area(t.box[c]);
                if(a > ba) { ba = a; best = int(i); }
            }
            if(best < 0) break;
            const uint32_t c = b.slots[size_t(best)];
            b.expanded.push_back(c);
            b.slots.erase(b.slots.begin() + best);
            b.slots.insert(b.slots.begin() + best, t.kids[c].begin(), t.kids[c].end());
        }
        return b;
    };
    if(t.leaf(0))
    {   // a one-leaf BVH: its block holds the leaf
        Blk b;
        b.root = 0;
        b.slots.push_back(0);
        blks.push_back(b);
    }
    else
        blks.push_back(make(0));
    for(size_t q = 0; q < blks.size(); ++q)            // breadth-first
    {
        block_of[blks[q].root] = block_base + uint32_t(out.size() / kBlockCopies + q);
        for(uint32_t c: std::vector<uint32_t>(blks[q].slots))
            if(!t.leaf(c)) blks.push_back(make(c));
    }
    if(uint64_t(block_base) + out.size() / kBlockCopies + blks.size() > kBeIndex)
    { err = "BVH records above 2^28 blocks"; return false; }
    if(out.size() % kBlockCopies) { err = "unaligned block output"; return false; }

    // stack bound: a block step walks one passing entry and pushes the
    // others (at most all but one); a walk holds at most one block's pushes
    // per level of its path
    std::vector<uint32_t> bound(blks.size(), 0);
    const uint32_t first = uint32_t(out.size() / kBlockCopies) + block_base;
    for(size_t q = blks.size(); q-- > 0;)
    {
        uint32_t own = uint32_t(blks[q].slots.size()) - 1u, below = 0;
        for(uint32_t c: blks[q].slots)
        {
            if(!t.leaf(c)) below = std::max(below, bound[block_of[c] - first]);   // children come later (BFS)
        }
        bound[q] = own + below;
    }

    for(const Blk& b: blks)
    {
        // one copy per octant o: the entries in the order a ray of that
        // octant meets them (depth-first through the expanded nodes, each
        // one's children forward or reversed by its axis, bvh.cc:177-181),
        // each box as (near planes, far planes) for that octant's signs
        for(uint32_t o = 0; o < 8; ++o)
        {
            std::vector<uint32_t> seq;
            seq.reserve(W);
            auto walk = [&](auto&& self, uint32_t n) -> void {
                const std::vector<uint32_t>& ks = t.kids[n];
                const bool rev = ((o >> t.axis[n]) & 1u) == 0;
                for(size_t j = 0; j < ks.size(); ++j)
                {
                    const uint32_t c = ks[rev ? ks.size() - 1 - j : j];
                    if(std::find(b.expanded.begin(), b.expanded.end(), c) != b.expanded.end()) self(self, c);
                    else seq.push_back(c);
                }
            };
            if(t.leaf(b.root)) seq.push_back(b.root);
            else walk(walk, b.root);
            if(seq.size() != b.slots.size() || seq.size() > W) { err = "block order lost an entry"; return false; }
            BlockCopy bc{};
            for(uint32_t j = 0; j < W; ++j)
            {
                if(j >= seq.size())
                {   // an unused slot: planes at +-inf such that, for a ray of this
                    // octant (its reciprocal's sign per axis is the octant's), the
                    // near plane's t is +inf and the far plane's -inf - it never
                    // passes the walker's clamped test (BlockWalker::box_near_far);
                    // the min/max form checks kBeNone
                    const float inf = std::numeric_limits<float>::infinity();
                    const bool px = o & 1u, py = o & 2u, pz = o & 4u;
                    bc.n[j] = BlockCopy::Near{px ? inf : -inf, py ? inf : -inf, pz ? inf : -inf, kBeNone};
                    bc.f[3 * j] = px ? -inf : inf;
                    bc.f[3 * j + 1] = py ? -inf : inf;
                    bc.f[3 * j + 2] = pz ? -inf : inf;
                    continue;
                }
                const uint32_t c = seq[j];
                const ptg_bvh_node& n = t.box[c];
                const bool px = o & 1u, py = o & 2u, pz = o & 4u;
                bc.n[j] = BlockCopy::Near{px ? n.min_x : n.max_x, py ? n.min_y : n.max_y, pz ? n.min_z : n.max_z,
                                          t.leaf(c) ? t.payload[c] : block_of[c]};
                bc.f[3 * j] = px ? n.max_x : n.min_x;
                bc.f[3 * j + 1] = py ? n.max_y : n.min_y;
                bc.f[3 * j + 2] = pz ? n.max_z : n.min_z;
            }
            out.push_back(bc);
        }
    }
    info.root = block_base + uint32_t((out.size() / kBlockCopies) - blks.size());
    info.blocks = uint32_t(blks.size());
    info.stack_entries = bound.empty() ? 0 : bound[0];
    info.max_payload = 0;
    for(uint32_t n = 0; n < count; ++n)
        if(t.leaf(n)) info.max_payload = std::max(info.max_payload, t.payload[n] & kBeIndex);
    return true;
}

} // namespace ptg

namespace ptg {

bool leaf_boxes_are_vertex_bounds(const ptg_bvh_node* nodes, const ptg_bvh_link* links, uint32_t count,
                                  const uint32_t* indices, size_t index_count, const ptg_float3* pos, size_t vertex_count,
                                  uint32_t index_offset, uint32_t triangle_count, uint32_t base_vertex_offset)
{
    for(uint32_t n = 0; n < count; ++n)
    {
        const ptg_bvh_link& l = links[n];   // octant 0's order
        if(!(l.accept & 0x80000000u)) continue;
        const uint32_t t = l.accept & 0x7FFFFFFFu;
        const size_t i0 = size_t(index_offset) + 3 * size_t(t);
        if(t >= triangle_count || i0 + 3 > index_count) return false;
        const ptg_float3* P[3];
        for(int k = 0; k < 3; ++k)
        {
            const size_t v = size_t(base_vertex_offset) + indices[i0 + k];
            if(v >= vertex_count) return false;
            P[k] = pos + v;
        }
        using hm::fminf_;
        using hm::fmaxf_;
        const float lo[3] = {fminf_(P[0]->x, fminf_(P[1]->x, P[2]->x)), fminf_(P[0]->y, fminf_(P[1]->y, P[2]->y)),
                             fminf_(P[0]->z, fminf_(P[1]->z, P[2]->z))};
        const float hi[3] = {fmaxf_(P[0]->x, fmaxf_(P[1]->x, P[2]->x)), fmaxf_(P[0]->y, fmaxf_(P[1]->y, P[2]->y)),
                             fmaxf_(P[0]->z, fmaxf_(P[1]->z, P[2]->z))};
        if(memcmp(lo, &nodes[n].min_x, 12) != 0 || memcmp(hi, &nodes[n].max_x, 12) != 0) return false;
    }
    return true;
}

// The subframes' TLASes are built over nearly the same instances (only the
// moving ones differ), so most of their subtrees are identical: ~98% of the
// blocks at 1024 spp.  Identical subtrees are stored once (hash-consing,
// children before parents): the trees, and so every walk, are unchanged,
// but the TLAS records shrink from ~51 MB to 1-2 MB and stay in L2.
static void dedup_tlas(FramePack& fp)
{
    const size_t E = kBlockCopies, nb = fp.tlas.size() / E;
    if(nb == 0) return;
    std::vector<uint32_t> canon(nb);
    std::vector<BlockCopy> uniq;   // distinct blocks, inner links as distinct-block ids
    std::unordered_map<uint64_t, std::vector<uint32_t>> table;
    BlockCopy tmp[kBlockCopies];
    for(size_t k = nb; k-- > 0;)
    {   // BFS within each TLAS: a block's children come after it
        memcpy(tmp, &fp.tlas[k * E], sizeof(tmp));
        for(BlockCopy& c: tmp)
            for(BlockCopy::Near& e: c.n)
                if(!(e.a & (kBeLeaf | kBeNone))) e.a = canon[e.a - fp.tlas_base];
        uint64_t h = 1469598103934665603ull;   // FNV-style mix over the block's 64-bit words
        static_assert(sizeof(tmp) % 8 == 0, "whole words");
        for(size_t i = 0; i < sizeof(tmp); i += 8)
        {
            uint64_t w;
            memcpy(&w, reinterpret_cast<const unsigned char*>(tmp) + i, 8);
            h = (h ^ w) * 1099511628211ull;
            h ^= h >> 29;
        }
        std::vector<uint32_t>& bucket = table[h];
        uint32_t id = 0xFFFFFFFFu;
        for(uint32_t c: bucket)
            if(!memcmp(&uniq[size_t(c) * E], tmp, sizeof(tmp))) { id = c; break; }
        if(id == 0xFFFFFFFFu)
        {
            id = uint32_t(uniq.size() / E);
            uniq.insert(uniq.end(), tmp, tmp + E);
            bucket.push_back(id);
        }
        canon[k] = id;
    }
    // lay the distinct blocks out in order of first use (the first TLAS's
    // breadth-first order, then what later subframes add)
    const uint32_t nu = uint32_t(uniq.size() / E);
    std::vector<uint32_t> pos(nu, 0xFFFFFFFFu);
    uint32_t next = 0;
    for(size_t k = 0; k < nb; ++k)
        if(pos[canon[k]] == 0xFFFFFFFFu) pos[canon[k]] = next++;
    std::vector<BlockCopy> out(size_t(nu) * E);
    for(uint32_t id = 0; id < nu; ++id)
        for(size_t j = 0; j < E; ++j)
        {
            BlockCopy c = uniq[size_t(id) * E + j];
            for(BlockCopy::Near& e: c.n)
                if(!(e.a & (kBeLeaf | kBeNone))) e.a = fp.tlas_base + pos[e.a];
            out[size_t(pos[id]) * E + j] = c;
        }
    for(uint32_t& r: fp.tlas_root) r = fp.tlas_base + pos[canon[r - fp.tlas_base]];
    fp.tlas.swap(out);
}

int BlockCache::pack_frame(const ptg_bvh_node* static_nodes, const ptg_bvh_link* static_links, size_t static_count,
                           size_t index_count, size_t vertex_count, const ptg_subframe* subframes, size_t subframe_count,
                           const ptg_tlas_instance* instances, size_t instance_count, const ptg_bvh_node* frame_nodes,
                           const ptg_bvh_link* frame_links, size_t first_node, size_t frame_node_count, FramePack& fp,
                           std::string& err) const
{
    fp = FramePack();
    fp.blas_base = uint32_t(blas.size() / kBlockCopies);
    fp.blas_stack = blas_stack;
    fp.inst_root.resize(instance_count);
    std::string why;
    for(size_t i = 0; i < instance_count; ++i)
    {
        const ptg_tlas_instance& in = instances[i];
        const std::string who = "instance " + std::to_string(i);
        if(uint64_t(in.blas.node_offset) + in.blas.node_count > static_count || in.blas.node_count == 0)
        { err = who + ": BLAS outside the static nodes"; return PTG_E_RANGE; }
        if(uint64_t(in.m.index_offset) + 3ull * in.m.triangle_count > index_count || in.m.index_offset % 3 ||
           uint64_t(in.m.base_vertex_offset) + in.m.vertex_count > vertex_count)
        { err = who + ": mesh outside the uploaded buffers"; return PTG_E_RANGE; }
        const uint32_t key = in.blas.node_offset;
        BlasRecord rec;
        if(auto o = records.find(key); o != records.end()) rec = o->second;
        else if(auto f = fp.new_records.find(key); f != fp.new_records.end()) rec = f->second;
        else
        {
            BlockBvh info;
            if(!pack_block_bvh(static_nodes + in.blas.node_offset, static_links + size_t(in.blas.node_offset) * 8,
                               in.blas.node_count, fp.blas_base, 1u << 28, fp.new_blas, info, why))
            { err = who + ": BLAS at node " + std::to_string(in.blas.node_offset) + ": " + why; return PTG_E_RANGE; }
            rec.root = info.root;
            rec.count = in.blas.node_count;
            rec.max_payload = info.max_payload;
            fp.new_records[key] = rec;
            fp.blas_stack = std::max(fp.blas_stack, info.stack_entries);
        }
        if(rec.count != in.blas.node_count) { err = who + ": BLAS node count differs from an earlier instance's"; return PTG_E_RANGE; }
        if(rec.max_payload >= in.m.triangle_count)
        {
            err = who + ": BLAS names triangle " + std::to_string(rec.max_payload) + " of a " +
                  std::to_string(in.m.triangle_count) + "-triangle mesh";
            return PTG_E_RANGE;
        }
        fp.inst_root[i] = rec.root;
    }
    fp.tlas_base = fp.blas_base + uint32_t(fp.new_blas.size() / kBlockCopies);
    fp.tlas_root.resize(subframe_count);
    for(size_t i = 0; i < subframe_count; ++i)
    {
        const ptg_bvh& t = subframes[i].tlas;
        if(t.node_offset < first_node || uint64_t(t.node_offset) + t.node_count > first_node + frame_node_count ||
           t.node_count == 0)
        { err = "subframe " + std::to_string(i) + ": TLAS outside the frame nodes"; return PTG_E_RANGE; }
    }
    // The subframes' TLASes are independent: packed on several host threads,
    // each at block base 0, then laid out one after another and relocated.
    std::vector<std::vector<BlockCopy>> part(subframe_count);
    std::vector<BlockBvh> pinfo(subframe_count);
    std::vector<std::string> perr(subframe_count);
    std::vector<char> pok(subframe_count, 0);
    auto pack_range = [&](size_t i0, size_t i1) {
        for(size_t i = i0; i < i1; ++i)
        {
            const ptg_bvh& t = subframes[i].tlas;
            const size_t rel = t.node_offset - first_node;
            // every TLAS leaf must name a valid instance
            pok[i] = pack_block_bvh(frame_nodes + rel, frame_links + 8 * rel, t.node_count, 0, uint32_t(instance_count),
                                    part[i], pinfo[i], perr[i]);
        }
    };
    const size_t nthreads = std::min<size_t>(subframe_count, std::min(8u, host_threads()));
    if(nthreads > 1)
    {
        std::vector<std::thread> pool;
        for(size_t k = 0; k < nthreads; ++k)
            pool.emplace_back(pack_range, subframe_count * k / nthreads, subframe_count * (k + 1) / nthreads);
        for(std::thread& th: pool) th.join();
    }
    else
        pack_range(0, subframe_count);
    size_t total_entries = 0;
    for(size_t i = 0; i < subframe_count; ++i)
    {
        if(!pok[i]) { err = "subframe " + std::to_string(i) + ": TLAS: " + perr[i]; return PTG_E_RANGE; }
        total_entries += part[i].size();
    }
    fp.tlas.reserve(total_entries);
    for(size_t i = 0; i < subframe_count; ++i)
    {
        const uint32_t base = fp.tlas_base + uint32_t(fp.tlas.size() / kBlockCopies);
        if(uint64_t(base) + part[i].size() / kBlockCopies > kBeIndex) { err = "TLAS records above 2^28 blocks"; return PTG_E_RANGE; }
        for(BlockCopy c: part[i])
        {
            for(BlockCopy::Near& e: c.n)
                if(!(e.a & (kBeLeaf | kBeNone))) e.a += base;
            fp.tlas.push_back(c);
        }
        fp.tlas_root[i] = pinfo[i].root + base;
        fp.tlas_stack = std::max(fp.tlas_stack, pinfo[i].stack_entries);
    }
    dedup_tlas(fp);
    // every block index a walk can follow lies inside the buffer (the
    // committed BLAS blocks were checked when they were added)
    const uint32_t total = fp.total_blocks();
    for(const std::vector<BlockCopy>* v: {&fp.new_blas, &fp.tlas})
        for(const BlockCopy& c: *v)
            for(const BlockCopy::Near& e: c.n)
                if(!(e.a & (kBeLeaf | kBeNone)) && e.a >= total) { err = "block link outside the block buffer"; return PTG_E_RANGE; }
    for(uint32_t r: fp.tlas_root)
        if(r >= total) { err = "TLAS root outside the block buffer"; return PTG_E_RANGE; }
    for(uint32_t r: fp.inst_root)
        if(r >= total) { err = "BLAS root outside the block buffer"; return PTG_E_RANGE; }
    return PTG_OK;
}

void BlockCache::commit(FramePack& fp)
{
    blas.insert(blas.end(), fp.new_blas.begin(), fp.new_blas.end());
    for(const auto& kv: fp.new_records) records[kv.first] = kv.second;
    blas_stack = fp.blas_stack;
}

} // namespace ptg
