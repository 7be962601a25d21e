// Device path tracer: the reference hot path re-expressed for gfx950.
//
//   trace()              two-level stackless BVH walk with the reference's
//                        link order (ray_query.hh:111-290) as ONE flat loop:
//                        TLAS and BLAS steps, BLAS entry and triangle tests
//                        are all iterations of the same loop, so lanes of a
//                        wave that sit in different levels still step
//                        together (no nested per-level loops to diverge in).
//   path_trace_sample()  path_trace_pixel (path_tracer.hh:637-741).
//   tonemap()            tonemap_pixel (path_tracer.hh:753-771).
//
// Results are bit-identical to the reference's C++ evaluated in IEEE
// arithmetic (oracle/pt_oracle.c): every float/double expression below keeps
// the reference's operand order and precision; see ref_math.h for the rules.
#pragma once
#include "layout.h"
#include "ref_math.h"

namespace ptg {
namespace dm {

constexpr float EARTH_RADIUS = 6.3781e6f;
constexpr float ATMOSPHERE_HEIGHT = 1.0e5f;
constexpr float RAYLEIGH_SCALE_HEIGHT = 7994.0f;
constexpr float MIE_SCALE_HEIGHT = 1200.0f;
// -height / scale height via div_by (== the IEEE division for every float, ref_math.h)
PTG_D float ray_h(float h) { return div_by(-h, RAYLEIGH_SCALE_HEIGHT, 1.0f / RAYLEIGH_SCALE_HEIGHT); }
PTG_D float mie_h(float h) { return div_by(-h, MIE_SCALE_HEIGHT, 1.0f / MIE_SCALE_HEIGHT); }
constexpr float MIE_ANISOTROPY = 0.80f;
constexpr float MIN_RAY_DIST = 1e-4f;
constexpr float MAX_RAY_DIST = 1e9f;
constexpr float REGULARIZATION_GAMMA = 0.15f;
constexpr int PRIMARY_ITERATIONS = 8;
constexpr int SECONDARY_ITERATIONS = 4;

// Work counters (only in the counting build of a kernel).
#if PTG_DEBUG
#define PTG_CHECK(sc, cond, slot)                                     \
    do {                                                              \
        if(!(cond))                                                   \
        {                                                             \
            if((sc).debug) atomicAdd((sc).debug + (slot), 1u);        \
            return 1;                                                 \
        }                                                             \
    } while(0)
#else
#define PTG_CHECK(sc, cond, slot) do {} while(0)
#endif

struct Counters {
    uint32_t visits = 0, tri_tests = 0, blas_entries = 0, queries = 0, shades = 0, tlas_visits = 0, iters = 0;
    uint32_t step_loads = 0;   // walk statistics: loads of the last step (1 block rows, 2 triangle, 4 instance)
};

struct Hit {
    float bx, by, bz, thit;
    uint32_t instance_id, primitive_id;
    bool back_face;
};

// the walk's reciprocals via rcp_rn (== 1.0f / x for every x, ref_math.h)
PTG_D float wrcp(float x) { return rcp_rn(x); }
PTG_D float rcp_or_big(float d) { return d == 0 ? __builtin_inff() : wrcp(d); }   // 1/d, 0 -> (float)1e40
PTG_D bool finite3(f3 v) { return __builtin_isfinite(v.x) && __builtin_isfinite(v.y) && __builtin_isfinite(v.z); }
PTG_D uint32_t octant(f3 d) { return (d.x > 0 ? 1u : 0u) | (d.y > 0 ? 2u : 0u) | (d.z > 0 ? 4u : 0u); }

// ray_triangle_intersection (math.hh:358-401) followed by the distance test of
// ray_query_test_triangle (ray_query.hh:243-245): true when the triangle
// P0 P1 P2 is an accepted candidate (det != 0, t >= 0, barycentrics of one
// sign, tmin < t < tmax); u, v, t and back are then the candidate's values.
// The division-free parts of the acceptance test come first: most tested
// triangles fail them and then skip the reciprocal.
PTG_D bool tri_accept(f3 org, int axis, f3 S, f3 P0, f3 P1, f3 P2, float tmin, float tmax, float& u, float& v,
                      float& t, bool& back)
{
    const f3 A = P0 - org, B = P1 - org, C = P2 - org;
    f3 x = V3(A.x, B.x, C.x), y = V3(A.y, B.y, C.y), z = V3(A.z, B.z, C.z);
    if(axis == 0) { x = z; z = V3(A.x, B.x, C.x); }
    else if(axis == 1) { y = z; z = V3(A.y, B.y, C.y); }
    x = x - S.x * z;
    y = y - S.y * z;
    const f3 uvw = cross(y, x);
    const float det = uvw.x + uvw.y + uvw.z;
    if(!(det != 0.0f && ((uvw.x >= 0.0f && uvw.y >= 0.0f && uvw.z >= 0.0f) ||
                         (uvw.x <= 0.0f && uvw.y <= 0.0f && uvw.z <= 0.0f))))
        return false;
    const float rdet = wrcp(det);
    u = uvw.x * rdet;
    v = uvw.y * rdet;
    t = dot(uvw, S.z * z) * rdet;
    back = det < 0;
    if(S.z < 0) back = !back;
    if(axis != 2) back = !back;
    return t >= 0.0f && t < tmax && t > tmin;
}

// ray_triangle_intersection_preprocess (math.hh:340-356)
PTG_D void tri_preprocess(f3 d, int& axis, f3& S)
{
    const float ax = fabsf(d.x), ay = fabsf(d.y), az = fabsf(d.z);
    f3 rd = d;
    axis = 2;
    if(ax > ay && ax > az) { axis = 0; rd = V3(d.z, d.y, d.x); }
    else if(ay > az) { axis = 1; rd = V3(d.x, d.z, d.y); }
    const float k = 1.0f / rd.z;
    S = V3(rd.x * k, rd.y * k, 1.0f * k);
}

// slab test of ray_query_traverse (ray_query.hh:197-207)
PTG_D bool slab_hit(f3 org, f3 inv, float tmin, float tmax, float lx, float ly, float lz, float hx, float hy, float hz)
{
    const float t0x = (lx - org.x) * inv.x, t1x = (hx - org.x) * inv.x;
    const float t0y = (ly - org.y) * inv.y, t1y = (hy - org.y) * inv.y;
    const float t0z = (lz - org.z) * inv.z, t1z = (hz - org.z) * inv.z;
    const float nearv = fmaxf(fminf(t0x, t1x), fmaxf(fminf(t0y, t1y), fminf(t0z, t1z)));
    const float farv = fminf(fmaxf(t0x, t1x), fminf(fmaxf(t0y, t1y), fmaxf(t0z, t1z)));
    return nearv <= farv && farv > tmin && nearv < tmax;
}

// Where a walk keeps its cold state - the world ray and the best hit so
// far.  They are touched only when a BLAS is entered or left and
// when a hit is confirmed, so a walker keeps them in registers (RegCold) or,
// where registers and LDS decide the occupancy, in a per-lane LDS slot
// (LdsCold, the wavefront walk kernels).
struct RegCold {
    f3 o, d;                   // world ray
    Hit best;

    PTG_D void init(f3 ro, f3 rd, f3)
    {
        o = ro; d = rd;
        best.thit = -1.0f;
        best.bx = best.by = best.bz = 0.0f;
        best.instance_id = 0xFFFFFFFFu;
        best.primitive_id = 0;
        best.back_face = false;
    }
    PTG_D f3 world_o() const { return o; }
    PTG_D f3 world_d() const { return d; }
    // any-hit occluder candidates are tried only by the wavefront walk (LdsCold)
    PTG_D uint32_t candidate_skip() const { return 0xFFFFFFFFu; }
    PTG_D uint32_t candidate_root() const { return kBePop; }
    PTG_D void set_candidate(uint32_t, uint32_t) {}
    PTG_D void clear_candidate_root() {}
    static constexpr bool kGlobalTri = false;   // confirm() takes the mesh-local primitive
    // ray_query_confirm (ray_query.hh:280-290)
    PTG_D void confirm(float u, float v, float t, uint32_t instance, uint32_t prim, bool back)
    {
        best.bx = u;
        best.by = v;
        best.bz = 1.0f - u - v;
        best.thit = t;
        best.instance_id = instance;
        best.primitive_id = prim;
        best.back_face = back;
    }
    PTG_D Hit result(float) const { return best; }
};

struct WalkCold {              // one lane's LDS slot: two b128 accesses
    float4 o;                  // world origin xyz; w: the any-hit candidate's instance (BlockWalker::try_candidate)
    float4 d;                  // world direction xyz; w: the TLAS root still to walk after it, or kBePop
};
// LDS (address space 3) pointers to clang vector types: accesses through
// them are ds_* instructions, never flat ones the compiler would have to
// route at run time (HIP's float4/uint2 classes cannot be assigned through
// an address-space pointer)
typedef float lds_f4v __attribute__((ext_vector_type(4)));
typedef uint32_t lds_u2v __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(3))) lds_f4v lds_cold_t;   // [0] = WalkCold::o, [1] = WalkCold::d
typedef __attribute__((address_space(3))) lds_u2v lds_uint2_t;

// World ray in LDS (read at BLAS entry and exit), best hit in registers.
struct LdsCold {
    lds_cold_t* c;
    float bu, bv;
    uint32_t binst, bprim;     // bprim: primitive | back_face << 31

    PTG_D void init(f3 ro, f3 rd, f3)
    {
        c[0] = lds_f4v{ro.x, ro.y, ro.z, __uint_as_float(0xFFFFFFFFu)};
        c[1] = lds_f4v{rd.x, rd.y, rd.z, __uint_as_float(kBePop)};
        bu = bv = 0.0f;
        binst = 0xFFFFFFFFu;
        bprim = 0;
    }
    // the any-hit candidate state sits in the w words of the world ray's rows,
    // read with them at BLAS entry and exit (no registers held across steps)
    PTG_D uint32_t candidate_skip() const { const lds_f4v v = c[0]; return __float_as_uint(v.w); }
    PTG_D uint32_t candidate_root() const { const lds_f4v v = c[1]; return __float_as_uint(v.w); }
    PTG_D void set_candidate(uint32_t inst, uint32_t root)
    {
        typedef __attribute__((address_space(3))) float lds_f_t;
        reinterpret_cast<lds_f_t*>(c)[3] = __uint_as_float(inst);
        reinterpret_cast<lds_f_t*>(c)[7] = __uint_as_float(root);
    }
    PTG_D void clear_candidate_root()
    {
        typedef __attribute__((address_space(3))) float lds_f_t;
        reinterpret_cast<lds_f_t*>(c)[7] = __uint_as_float(kBePop);
    }
    // confirm() takes the BLAS's triangle base + the primitive (the TriRec /
    // TriShade index), which the wavefront hit record carries to the shading
    static constexpr bool kGlobalTri = true;
    PTG_D f3 world_o() const { const lds_f4v v = c[0]; return V3(v.x, v.y, v.z); }
    PTG_D f3 world_d() const { const lds_f4v v = c[1]; return V3(v.x, v.y, v.z); }
    // ray_query_confirm (ray_query.hh:280-290); thit is the walk's tmax, bz is
    // derived in result() with the same arithmetic
    PTG_D void confirm(float u, float v, float, uint32_t instance, uint32_t prim, bool back)
    {
        bu = u;
        bv = v;
        binst = instance;
        bprim = prim | (back ? 0x80000000u : 0u);
    }
    PTG_D Hit result(float tmax) const
    {
        const bool hit = binst != 0xFFFFFFFFu;
        Hit h;
        h.bx = bu;
        h.by = bv;
        h.bz = hit ? 1.0f - bu - bv : 0.0f;
        h.thit = hit ? tmax : -1.0f;
        h.instance_id = binst;
        h.primitive_id = bprim & 0x7FFFFFFFu;
        h.back_face = (bprim >> 31) != 0;
        return h;
    }
};

// Per-lane walk stacks of (word, near) entries (block_format.h: word = a
// block index or kBeLeaf | payload; near = the entry distance, re-checked
// against tmax when the entry is popped).
// PrivStack: a private array (scratch memory) for the per-lane megakernel and
// the per-ray entry points; the host checks every frame's stack bound
// against kCap before those kernels run.
struct PrivStack {
    static constexpr uint32_t kCap = kBlockWidth > 4 ? 128 : 96;   // entries; put() may write one past the bound
    uint2 v[kCap];
    uint32_t sp;
    PTG_D void reset() { sp = 0; }
    PTG_D uint32_t size() const { return sp; }
    PTG_D void reserve(uint32_t) {}
    PTG_D void put(uint2 e, bool keep) { v[sp] = e; sp += keep ? 1u : 0u; }
    PTG_D uint2 pop() { return v[--sp]; }
    PTG_D bool fits(uint32_t n, uint32_t stride) const { return sp + n <= stride; }
};

// LdsStack: the wavefront walks' stack.  The newest entries of a lane live
// in LDS, in a window of kCap slots (one 8-byte column per lane: slot k of a
// wave's 64 lanes is one conflict-free 512 B row), addressed through a
// pointer to the next free slot, so a push is one ds_write at that pointer
// and a pointer bump.  When a block step could overflow the window, its
// oldest half goes to the lane's area in HBM and the rest moves down (rare);
// those entries come back one by one when the stack unwinds to them.  A
// 16-entry window holds the whole stack for all but ~0.03 entries per query
// of a heavy frame.
#ifndef PTG_STACK_ENTRIES
#define PTG_STACK_ENTRIES 16
#endif
struct LdsStack {
    static constexpr uint32_t kCap = PTG_STACK_ENTRIES;
    lds_uint2_t* s;            // the lane's window column: slot k at s[64 * k]
    lds_uint2_t* t;            // next free slot: s + 64 * (sp - lo)
    uint2* g;                  // the lane's spill area (HBM)
    uint32_t sp, lo;           // entries; entries below lo are in HBM
    static constexpr uint32_t kLaneBytes = 8u * kCap;   // LDS per lane
    // windows: one 64-lane x kCap table per wave from `lds` on; `spill`: the lane's area
    PTG_D void bind(void* lds, uint32_t wave, uint32_t lane, uint2* spill)
    {
        s = (lds_uint2_t*)(reinterpret_cast<uint2*>(lds) + wave * (64u * kCap) + lane);   // C cast: generic -> LDS
        g = spill;
    }
    PTG_D void reset()
    {
        sp = lo = 0;
        t = s;
    }
    PTG_D uint32_t size() const { return sp; }
    // room for n more entries in the window (rare: spill the oldest half)
    PTG_D void reserve(uint32_t n)
    {
        if(sp - lo + n <= kCap) return;
        const uint32_t in = sp - lo, h = in > 1 ? in / 2 : in;
        for(uint32_t i = 0; i < h; ++i)
        {
            const lds_u2v v = s[64u * i];
            g[lo + i] = make_uint2(v.x, v.y);
        }
        for(uint32_t i = h; i < in; ++i) s[64u * (i - h)] = s[64u * i];
        lo += h;
        t = s + 64u * (sp - lo);
    }
    // write e at the top; keep it (push) iff `keep`
    PTG_D void put(uint2 e, bool keep)
    {
        *t = lds_u2v{e.x, e.y};
        if(keep)
        {
            t += 64;
            ++sp;
        }
    }
    PTG_D uint2 pop()
    {
        --sp;
        if(sp < lo)
        {   // the window is empty: the entry comes back from HBM
            lo = sp;
            return g[sp];
        }
        t -= 64;
        const lds_u2v v = *t;
        return make_uint2(v.x, v.y);
    }
    // whether n more entries fit the lane's spill area of `stride` entries (PTG_DEBUG)
    PTG_D bool fits(uint32_t n, uint32_t stride) const { return sp + n <= stride; }
};

// The wavefront walks' stack: 4-byte slots (LdsSlotStack), or (word, near)
// pairs (LdsStack, PTG_SLOT_STACK=0).  Window sizes in slots: 24 for the
// closest-hit walk (a leaf takes two), 16 for the any-hit walk (one each).
#ifndef PTG_SLOT_STACK
#define PTG_SLOT_STACK 2
#endif
#ifndef PTG_STACK_SLOTS
#define PTG_STACK_SLOTS 24
#endif
#ifndef PTG_STACK_SLOTS_ANY
#define PTG_STACK_SLOTS_ANY 16
#endif
// LdsSlotStack: the same window in 4-byte slots (half the LDS per entry, so
// more walk blocks fit a CU).  A block entry is one slot, its word: its near
// need not be kept, because a block whose re-check at the pop would fail
// holds only children that fail too (block_format.h, fact 1: their near is at
// least the block's), so stepping it merely costs a block step.  A leaf entry
// keeps its near - the leaf's own box test at its own time (fact 2) - in a
// second slot under its word: NEAR = true (the closest-hit walk).  The
// any-hit walk's tmax never shrinks, so every pushed entry passes its re-check
// again at the pop (trace_shadow_ray: no ray_query_confirm): NEAR = false
// keeps words only.  The word is always on top, so a pop reads the top two
// slots with one ds_read2_b32 and takes the second only for a leaf.  Pushed
// nears are positive floats (the clamped entry distance, node_block), so a
// slot with the top bit set is always a leaf word, and a spill keeps leaf
// entries whole by looking at the slot above its cut.
template<bool NEAR>
struct LdsSlotStack {
    static constexpr uint32_t kCap = NEAR ? PTG_STACK_SLOTS : PTG_STACK_SLOTS_ANY;   // slots in the window
    typedef __attribute__((address_space(3))) uint32_t lds_u32_t;
    lds_u32_t* s;              // the lane's window column: slot k at s[64 * k]
    lds_u32_t* t;              // next free slot: s + 64 * (sp - lo)
    uint32_t* g;               // the lane's spill area (HBM), in slots
    uint32_t sp, lo;           // slots; slots below lo are in HBM
    static constexpr uint32_t kLaneBytes = 4u * kCap;   // LDS per lane
    PTG_D void bind(void* lds, uint32_t wave, uint32_t lane, uint2* spill)
    {
        s = (lds_u32_t*)(reinterpret_cast<uint32_t*>(lds) + wave * (64u * kCap) + lane);   // C cast: generic -> LDS
        g = reinterpret_cast<uint32_t*>(spill);
    }
    PTG_D void reset()
    {
        sp = lo = 0;
        t = s;
    }
    PTG_D uint32_t size() const { return sp; }
    // whether n more entries fit the lane's spill area of `stride` 8-byte
    // entries, i.e. 2 * stride slots (PTG_DEBUG)
    PTG_D bool fits(uint32_t n, uint32_t stride) const { return sp + (NEAR ? 2u : 1u) * n <= 2u * stride; }
    // room for n more entries in the window (rare: spill the oldest half)
    PTG_D void reserve(uint32_t n)
    {
        // put() writes two slots from the top whatever it keeps
        if(sp - lo + (NEAR ? 2u * n : n) <= kCap) return;
        const uint32_t in = sp - lo;
        uint32_t h = in > 1 ? in / 2 : in;
        if(NEAR && h < in && (s[64u * h] & kBeLeaf)) ++h;   // slot h - 1 is that leaf word's near: keep them together
        for(uint32_t i = 0; i < h; ++i) g[lo + i] = s[64u * i];
        for(uint32_t i = h; i < in; ++i) s[64u * (i - h)] = s[64u * i];
        lo += h;
        t = s + 64u * (sp - lo);
    }
    // write the entry at the top; keep it (push) iff `keep`
    PTG_D void put(uint2 e, bool keep)
    {
        if(NEAR)
        {
            const bool leaf = (e.x & kBeLeaf) != 0;
            t[0] = leaf ? e.y : e.x;
            t[64] = e.x;
            const uint32_t k = keep ? (leaf ? 2u : 1u) : 0u;
            t += 64u * k;
            sp += k;
        }
        else
        {
            t[0] = e.x;
            if(keep)
            {
                t += 64;
                ++sp;
            }
        }
    }
    // (word, near); a block's near reads as +0, which passes any tmax (tmax > 0)
    PTG_D uint2 pop()
    {
        if(sp == lo)
        {   // the window is empty: the entry comes back from HBM (rare)
            const uint32_t w = g[sp - 1];
            const bool leaf = NEAR && (w & kBeLeaf) != 0;
            const uint32_t n = leaf ? g[sp - 2] : 0u;
            sp -= leaf ? 2u : 1u;
            lo = sp;
            t = s;
            return make_uint2(w, n);
        }
        if(!NEAR)
        {
            --sp;
            t -= 64;
            return make_uint2(*t, 0u);
        }
        // one ds_read2_b32 (the slot under the window's bottom, read for a
        // block, is LDS of this block and unused)
        const uint32_t w = t[-64], n = t[-128];
        const bool leaf = (w & kBeLeaf) != 0;
        const uint32_t k = leaf ? 2u : 1u;
        t -= 64u * k;
        sp -= k;
        return make_uint2(w, leaf ? n : 0u);
    }
};

// PTG_SLOT_STACK bit 0: the closest-hit walk on slots, bit 1: the any-hit walk
template<bool ANY, bool SLOTS = ((PTG_SLOT_STACK >> (ANY ? 1 : 0)) & 1) != 0> struct WalkStackOf {
    typedef LdsStack type;
};
template<bool ANY> struct WalkStackOf<ANY, true> {
    typedef LdsSlotStack<!ANY> type;
};

// x_t for t in 0..3, as two selects on t's bits: by value, so that the
// compiler emits v_cndmask and neither branches nor indexes a stack copy
PTG_D uint32_t sel4(uint32_t t, uint32_t x0, uint32_t x1, uint32_t x2, uint32_t x3)
{
    const uint32_t lo = (t & 1u) ? x1 : x0;
    const uint32_t hi = (t & 1u) ? x3 : x2;
    return (t & 2u) ? hi : lo;
}

// One ray query over the block records (block_format.h), resumable: a step
// is one 4-wide block (node_step, which first pops the next stack entry if
// the walk needs one), or one triangle test or BLAS entry (leaf_step), of
// either level - so the lanes of a wave step together whatever level each
// is in, and a persistent kernel can swap rays between steps.  ANY = true is
// trace_shadow_ray (path_tracer.hh:415-427): the first accepted candidate
// ends the walk.  ANY = false is the proceed/confirm loop of trace_ray
// (path_tracer.hh:342-349): every accepted candidate is confirmed and
// shortens tmax.  Candidates are met in the reference's order with the
// reference's tmax (block_format.h), so the result is bit-identical to the
// reference's stackless link walk (ray_query.hh:184-278).
template<class Cold, class Stack>
struct BlockWalker {
    Cold cold;                 // world ray, best hit
    Stack st;
    float tmin, tmax;
    f3 org, inv;               // active level: ray origin / 1/dir in that level's space
    f3 winv;                   // the world ray's 1/dir (the TLAS level's inv)
    bool fin;                  // active level: every component of inv finite (box_near_far applies)
    uint32_t oct;              // active level: direction octant (the links' order index, ray_query.hh:139-140)
    f3 S;                      // BLAS: shear constants of ray_triangle_intersection_preprocess
    int axis;                  // BLAS: dominant axis, -1 while in the TLAS (blas_axis)
    uint32_t tri_base, inst, bsp;
    uint32_t cur;              // next block, leaf word, or kBePop
    float cnear;               // cur's entry distance (a leaf's is re-checked when it is tested)
    uint32_t pend;             // a parked triangle (leaf word), or kBePop
    float pnear;               // its entry distance

    // ray_query_initialize (ray_query.hh:111-151); root = the TLAS's root
    // block, kBePop for no TLAS (the walk ends at its first step)
    PTG_D void init(uint32_t root, f3 ro, f3 rd, float t0, float t1)
    {
        const f3 iw = V3(rcp_or_big(rd.x), rcp_or_big(rd.y), rcp_or_big(rd.z));
        cold.init(ro, rd, iw);
        tmin = t0;
        tmax = t1;
        org = ro;
        inv = iw;
        winv = iw;
        fin = finite3(iw);
        oct = octant(rd);
        S = V3(0, 0, 0);
        axis = -1;
        tri_base = 0;
        inst = 0xFFFFFFFFu;
        bsp = 0;
        st.reset();
        cur = root;
        cnear = -__builtin_inff();
        pend = kBePop;
        pnear = 0.0f;
    }

    // Any hit only (trace_shadow_ray, path_tracer.hh:415-427): the walk returns
    // whether ANY triangle passes its TLAS leaf box, its BLAS leaf box and its
    // triangle test - tmax never shrinks (no ray_query_confirm), so by
    // containment (block_format.h) the ancestors pass too, and the order in
    // which leaves are met does not change the result.  A candidate (instance
    // ci, triangle cp of its mesh - where a nearby ray found its occluder) is
    // therefore met first: ci's TLAS leaf box is tested here against its
    // InstBox (the reference's leaf node; ci must be a leaf of this ray's
    // subframe's TLAS), its BLAS is entered and walked whole with cp parked
    // first (cp's leaf box, its vertex bounds, tested with the triangle), and
    // then the TLAS from its root with ci's leaf skipped (ci held no
    // occluder).  Call right after init().  The instance to skip and the TLAS
    // root still to walk live in the cold state (Cold::set_candidate), the
    // candidate triangle in pend (flag kBeCand; a parked triangle waits for
    // the BLAS entry, leaf_select).  A walk that returns 2 leaves the
    // occluding triangle in cur.
    PTG_D void try_candidate(const DevScene& sc, uint32_t ci, uint32_t cp, uint32_t sub)
    {
        if(ci >= sc.inst_count || cur == kBePop) return;
        const float4* b = reinterpret_cast<const float4*>(sc.inst_box + ci);
        const float4 lo = b[0], hi = b[1];
        const uint32_t in = __float_as_uint(lo.w);
        float nv;
        if((in != sub && in != kInstAllSubframes) || cp >= __float_as_uint(hi.w) || !box(lo, hi, nv)) return;
        cold.set_candidate(ci, cur);
        cur = kBeLeaf | ci;
        cnear = nv;
        pend = kBeLeaf | kBeCand | cp;
        pnear = -__builtin_inff();
    }
    // When a walk with a candidate ends (node step returned 1: the stack is
    // empty and the walk is back at the TLAS level), the candidate's instance
    // has been walked whole without an occluder: the walk goes on over the
    // TLAS from its root, skipping that instance's leaf.  Returns whether it
    // goes on.
    PTG_D bool resume_tlas()
    {
        const uint32_t root = cold.candidate_root();
        if(root == kBePop) return false;
        cur = root;
        cnear = -__builtin_inff();
        cold.clear_candidate_root();
        return true;
    }
    PTG_D Hit result() const { return cold.result(tmax); }

    // slab test (ray_query.hh:197-207) with its entry distance
    PTG_D bool box(float4 lo, float4 hi, float& nearv) const
    {
        const float t0x = (lo.x - org.x) * inv.x, t1x = (hi.x - org.x) * inv.x;
        const float t0y = (lo.y - org.y) * inv.y, t1y = (hi.y - org.y) * inv.y;
        const float t0z = (lo.z - org.z) * inv.z, t1z = (hi.z - org.z) * inv.z;
        nearv = fmaxf(fminf(t0x, t1x), fmaxf(fminf(t0y, t1y), fminf(t0z, t1z)));
        const float farv = fminf(fmaxf(t0x, t1x), fminf(fmaxf(t0y, t1y), fmaxf(t0z, t1z)));
        return nearv <= farv && farv > tmin && nearv < tmax;
    }

    // The same test on a box stored as (near planes, far planes) for the
    // ray's octant, for a level whose 1/dir is finite in every component:
    // then t of the near plane IS fmin(t0, t1) of the reference's per-axis
    // pair (the product of the ordered differences with a finite nonzero
    // reciprocal keeps their order; equal values are equal), so the per-axis
    // min/max drop out.
    //
    // The three compares become one by clamping the interval: with tmin >= 0,
    // tmax > 0 finite, tmin_p the float after tmin and tmax_m the one before
    // tmax (integer +-1 on the bits; f32 denormals are kept, so the compares
    // see them exactly),
    //   near <= far && far > tmin && near < tmax
    //     <=>  max(near, tmin_p) <= min(far, tmax_m)   whenever tmin_p <= tmax_m,
    // and the returned entry distance max(near, tmin_p) re-checks at its pop
    // as near does: max(near, tmin_p) < tmax <=> near < tmax whenever
    // tmin_p < tmax.  When tmax <= tmin_p no float t has tmin < t < tmax, so
    // no triangle can be accepted any more and which boxes pass changes
    // nothing.  No NaN arises (finite planes, finite reciprocals); an unused
    // slot's planes are +-inf so that its near is +inf and its far -inf
    // (host/block_bvh.cpp), which fails.
    PTG_D bool box_near_far(float4 nr, float4 fr, float tmin_p, float tmax_m, float& nearv) const
    {
        const float tnx = (nr.x - org.x) * inv.x, tfx = (fr.x - org.x) * inv.x;
        const float tny = (nr.y - org.y) * inv.y, tfy = (fr.y - org.y) * inv.y;
        const float tnz = (nr.z - org.z) * inv.z, tfz = (fr.z - org.z) * inv.z;
        nearv = fmaxf(fmaxf(tnx, tmin_p), fmaxf(tny, tnz));
        const float farv = fminf(fminf(tfx, tmax_m), fminf(tfy, tfz));
        return nearv <= farv;
    }

    // ray_query_enter_blas (ray_query.hh:153-182) with instance `leaf`'s record:
    // rows M0..M3 of inv_transform in xyz; w: BLAS root block, triangle base
    typedef float v4f __attribute__((ext_vector_type(4)));
    PTG_D void enter(uint32_t leaf, v4f a, v4f b, v4f c, v4f e)
    {
        const f3 M0 = V3(a.x, a.y, a.z), M1 = V3(b.x, b.y, b.z), M2 = V3(c.x, c.y, c.z), M3 = V3(e.x, e.y, e.z);
        const f3 o = cold.world_o(), d = cold.world_d();
        org = V3(M0.x * o.x + M1.x * o.y + M2.x * o.z + M3.x * 1.0f,
                 M0.y * o.x + M1.y * o.y + M2.y * o.z + M3.y * 1.0f,
                 M0.z * o.x + M1.z * o.y + M2.z * o.z + M3.z * 1.0f);
        const f3 bd = V3(M0.x * d.x + M1.x * d.y + M2.x * d.z,
                         M0.y * d.x + M1.y * d.y + M2.y * d.z,
                         M0.z * d.x + M1.z * d.y + M2.z * d.z);
        cur = __float_as_uint(a.w);
        tri_base = __float_as_uint(b.w);
        inst = leaf;
        bsp = st.size();
        oct = octant(bd);
        bool ok = true;   // one fallback branch for the four reciprocals of the entry
        inv = V3(rcp_nr(bd.x, ok), rcp_nr(bd.y, ok), rcp_nr(bd.z, ok));
        // ray_triangle_intersection_preprocess (math.hh:340-356)
        const float ax = fabsf(bd.x), ay = fabsf(bd.y), az = fabsf(bd.z);
        f3 rd = bd;
        axis = 2;
        if(ax > ay && ax > az) { axis = 0; rd = V3(bd.z, bd.y, bd.x); }
        else if(ay > az) { axis = 1; rd = V3(bd.x, bd.z, bd.y); }
        float k = rcp_nr(rd.z, ok);
        if(!ok)
        {   // a zero, denormal or huge component (rare): IEEE division
            inv = V3(rcp_or_big(bd.x), rcp_or_big(bd.y), rcp_or_big(bd.z));
            k = 1.0f / rd.z;
        }
        S = V3(rd.x * k, rd.y * k, 1.0f * k);
        fin = finite3(inv);
    }

    // ray_query_test_triangle + ray_triangle_intersection (ray_query.hh:225-246,
    // math.hh:358-401) with triangle `leaf`'s TriRec chunks
    template<bool ANY>
    PTG_D int tri_test(uint32_t leaf, float4 q0, float4 q1, float4 q2)
    {
        float u, v, t;
        bool back;
        if(tri_accept(org, axis, S, V3(q0.x, q0.y, q0.z), V3(q0.w, q1.x, q1.y), V3(q1.z, q1.w, q2.x), tmin, tmax, u, v, t,
                      back))
        {
            if(ANY)
            {
                cur = leaf;   // the occluder, for the caller (the walk has ended)
                return 2;
            }
            cold.confirm(u, v, t, inst, Cold::kGlobalTri ? tri_base + leaf : leaf, back);
            tmax = t;
        }
        return 0;
    }

    PTG_D bool at_leaf() const { return (cur & kBeLeaf) && cur != kBePop; }
    // whether the leaf phase has work: a parked triangle, or a leaf in cur
    PTG_D bool wants_leaf() const { return pend != kBePop || at_leaf(); }

    // A triangle the walk reaches is parked (with its near) while
    // the walk goes on with its next node steps; the leaf phase tests it.
    // Triangles are still tested in the walk's order, each after a near <
    // tmax re-check at its own time, and tmax changes only at triangle tests:
    // the node steps taken meanwhile use a tmax that is, at worst, too large,
    // which only adds work (block_format.h, facts 1 and 2).  BLAS entries are
    // never parked, and a walk with a parked triangle does not leave its BLAS.
    PTG_D void park()
    {
        if(axis >= 0 && pend == kBePop && at_leaf())
        {
            pend = cur;
            pnear = cnear;
            cur = kBePop;
        }
    }

    // Node phase, first half: pop the next entry if the walk needs one.
    // Returns -1 when cur is a block to step now, else what node_step returns
    // (0: nothing to step this phase, 1: the walk has ended).
    PTG_D int node_pop()
    {
        if(cur != kBePop) return -1;
        // one pop per node phase: a culled entry or a parked triangle simply
        // costs the lane its phase.  Straight-line selects after the pop (no
        // nested early returns: the compiler turned each into exec-mask
        // bookkeeping on every lane)
        if(st.size() == (axis < 0 ? 0u : bsp))
        {   // this level's entries are exhausted (rare)
            if(axis < 0) return 1;
            if(pend != kBePop) return 0;   // its parked triangle needs this BLAS: wait for the leaf phase
            // BLAS exhausted: back to the TLAS (ray_query.hh:273-274)
            axis = -1;
            org = cold.world_o();
            inv = winv;
            fin = finite3(winv);
            oct = octant(cold.world_d());
            if(st.size() == 0) return 1;   // (ANY: resume_tlas may go on)
        }
        const uint2 e = st.pop();
        const float n = __uint_as_float(e.y);
        const bool live = n < tmax;                        // the entry's test at its own time
        const bool leaf = (e.x & kBeLeaf) != 0;
        const bool parked = live && leaf && axis >= 0 && pend == kBePop;   // park() of the popped triangle
        pend = parked ? e.x : pend;
        pnear = parked ? n : pnear;
        cur = live && !parked ? e.x : kBePop;
        cnear = n;
        return live && !leaf ? -1 : 0;                     // a block to step now, else nothing this phase
    }

    // this octant's copy of block cur: its kBlockWidth entries in the order
    // the ray meets them, each box as (near planes, far planes) for the
    // octant's signs; kBlockRows 16-byte rows (seven at width 4)
    static constexpr uint32_t kBlockRows = (28u * kBlockWidth + 15u) / 16u;
    PTG_D const v4f* block_rows(const DevScene& sc) const
    {   // a 32-bit byte offset from the buffer's base (the upload keeps the
        // block buffer below 4 GB), so the loads take the scalar-base +
        // vector-offset form instead of 64-bit address arithmetic per lane
        const uint32_t off = (cur * kBlockCopies + oct) * uint32_t(sizeof(BlockCopy));
        return reinterpret_cast<const v4f*>(reinterpret_cast<const uint8_t*>(sc.blocks) + off);
    }
    // float k of the packed far planes (rows kBlockWidth..): entry j's at 3j..3j+2
    static PTG_D float far_plane(const v4f* q, uint32_t k)
    {
        const v4f r = q[kBlockWidth + k / 4u];
        const uint32_t c = k % 4u;
        return c == 0 ? r.x : c == 1 ? r.y : c == 2 ? r.z : r.w;
    }

    // Node phase, second half: the block step on its rows.
    template<bool COUNT>
    PTG_D int node_block(const DevScene& sc, Counters& cnt, const v4f (&q)[kBlockRows])
    {
        // rows 0..W-1: entry j's near planes and word; then the far planes, packed
        constexpr uint32_t W = kBlockWidth;
        float4 l[W], h[W];
        uint32_t a[W];
        float nr[W];
#pragma unroll
        for(uint32_t j = 0; j < W; ++j)
        {
            l[j] = make_float4(q[j].x, q[j].y, q[j].z, q[j].w);
            h[j] = make_float4(far_plane(q, 3 * j), far_plane(q, 3 * j + 1), far_plane(q, 3 * j + 2), 0.0f);
            a[j] = __float_as_uint(l[j].w);
        }
        if(COUNT) cnt.step_loads |= 1u;
        // bit j: the entry the ray meets j-th passed.  Built inside each form's
        // branch, so the two branches merge an integer, not four lane masks
        // (a merge of lane masks costs exec-masked scalar and/or per mask)
        uint32_t hits = 0;
        if(__all(fin))
        {   // every lane's reciprocal finite (the rule): no per-axis min/max
            const float tmin_p = __uint_as_float(__float_as_uint(tmin) + 1u);
            const float tmax_m = __uint_as_float(__float_as_uint(tmax) - 1u);
#pragma unroll
            for(uint32_t j = 0; j < W; ++j) hits |= box_near_far(l[j], h[j], tmin_p, tmax_m, nr[j]) ? (1u << j) : 0u;
        }
        else
        {   // a lane with a zero or denormal direction component: the
            // reference's min/max form (an unordered pair gives the same);
            // an infinite reciprocal can pass an unused slot's infinite planes.
            // The entry distance is clamped as in the other form: max(near,
            // tmin_p) < tmax <=> near < tmax whenever tmin_p < tmax, and a
            // walk's tmax is never below tmin_p (the initial tmax, or a
            // confirmed t > tmin); at tmax == tmin_p no triangle can be
            // accepted any more.  A pushed near is then a positive float
            // (LdsSlotStack tells its slots from leaf words by the top bit).
            const float tmin_p = __uint_as_float(__float_as_uint(tmin) + 1u);
#pragma unroll
            for(uint32_t j = 0; j < W; ++j)
            {
                hits |= (box(l[j], h[j], nr[j]) && !(a[j] & kBeNone)) ? (1u << j) : 0u;
                nr[j] = fmaxf(nr[j], tmin_p);
            }
        }
        if(COUNT)
        {
            uint32_t tested = 0;
#pragma unroll
            for(uint32_t j = 0; j < W; ++j) tested += !(a[j] & kBeNone);
            cnt.visits += tested;
            if(axis < 0) cnt.tlas_visits += tested;
        }
        // The first entry that passed is walked next; the others are pushed
        // last-first, so they pop in order.
        const uint32_t first = uint32_t(__builtin_ctz(hits | (1u << W))) & (W - 1u);
        uint32_t fa, fn;   // entry `first`, by value (v_cndmask): neither a branch nor an indexed copy
        if constexpr(W == 4)
        {
            fa = sel4(first, a[0], a[1], a[2], a[3]);
            fn = sel4(first, __float_as_uint(nr[0]), __float_as_uint(nr[1]), __float_as_uint(nr[2]),
                      __float_as_uint(nr[3]));
        }
        else
        {
            fa = a[0];
            fn = __float_as_uint(nr[0]);
#pragma unroll
            for(uint32_t j = 1; j < W; ++j)
            {
                fa = first == j ? a[j] : fa;
                fn = first == j ? __float_as_uint(nr[j]) : fn;
            }
        }
        cur = hits ? fa : kBePop;
        cnear = __uint_as_float(fn);
        const uint32_t rest = hits & (hits - 1u);
        if(rest)
        {   // written at the top either way, kept only if pushed
            // (the host's stack bound, which sizes the spill areas, must hold)
            PTG_CHECK(sc, st.fits(uint32_t(__builtin_popcount(rest)), sc.spill_stride), kDebugStack);
            st.reserve(W - 1);
#pragma unroll
            for(uint32_t j = W - 1; j >= 1; --j) st.put(make_uint2(a[j], __float_as_uint(nr[j])), (rest >> j) & 1u);
        }
        park();
        return 0;
    }

    // Node phase: pop the next entry if the walk needs one, then, if it is a
    // block, one block step.  Returns 1 when the walk has ended, else 0 (the
    // walk may then stand at a leaf, which leaf_step() takes).
    template<bool COUNT>
    PTG_D int node_step(const DevScene& sc, Counters& cnt)
    {
        if(const int r = node_pop(); r >= 0) return r;
        PTG_CHECK(sc, cur < sc.block_count, kDebugNode);
        const v4f* p = block_rows(sc);
        v4f q[kBlockRows];
#pragma unroll
        for(uint32_t k = 0; k < kBlockRows; ++k) q[k] = p[k];
        return node_block<COUNT>(sc, cnt, q);
    }

    // Leaf phase, first half: the parked triangle, else the BLAS entry or
    // triangle the walk stands at; its record's rows and whether it is
    // tested (a triangle's box test at its own time: the walk re-checks near).
    struct LeafSel {
        const v4f* p;
        uint32_t id;
        bool parked, inst_leaf, tri, cand;
    };
    template<bool ANY = false>
    PTG_D LeafSel leaf_select(const DevScene& sc)
    {
        LeafSel ls;
        // (ANY: a candidate triangle is parked before its instance is entered,
        // try_candidate; it waits until the walk is in that BLAS)
        ls.parked = pend != kBePop && (!ANY || axis >= 0);
        ls.cand = ls.parked && (pend & kBeCand) != 0;   // a candidate triangle: its leaf box is still to test
        ls.id = (ls.parked ? pend : cur) & kBeIndex;
        const float n = ls.parked ? pnear : cnear;
        if(ls.parked) pend = kBePop;
        else cur = kBePop;
        ls.inst_leaf = !ls.parked && axis < 0;
        ls.tri = !ls.inst_leaf && n < tmax;
        // 32-bit byte offsets (the triangle records stay below 4 GB: checked
        // at upload) instead of 64-bit multiplies per lane
        const uint8_t* base = ls.inst_leaf ? reinterpret_cast<const uint8_t*>(sc.inst_trav)
                                           : reinterpret_cast<const uint8_t*>(sc.tris);
        const uint32_t off = ls.inst_leaf ? ls.id * uint32_t(sizeof(InstTrav)) : (tri_base + ls.id) * uint32_t(sizeof(TriRec));
        ls.p = reinterpret_cast<const v4f*>(base + off);
        return ls;
    }

    // Leaf phase, second half, on the record's first four rows.
    template<bool ANY, bool COUNT>
    PTG_D int leaf_finish(const DevScene& sc, Counters& cnt, const LeafSel& ls, v4f r0, v4f r1, v4f r2, v4f r3)
    {
        if(COUNT)
        {
            if(ls.inst_leaf) { cnt.blas_entries++; cnt.step_loads |= 4u; }
            if(ls.tri) { cnt.tri_tests++; cnt.step_loads |= 2u; }
        }
        if(ls.inst_leaf)
        {
            // the TLAS walk after a candidate's instance (try_candidate) skips it
            if(ANY && ls.id == cold.candidate_skip() && cold.candidate_root() == kBePop) return 0;
            enter(ls.id, r0, r1, r2, r3);
            return 0;
        }
        bool in_box = true;
        if(ANY && ls.cand)
        {   // a candidate's BLAS leaf box: its vertex bounds (bvh.cc:243-246: fmin / fmax
            // of the three positions; the upload checked every leaf box of this BLAS is)
            const float4 lo = make_float4(gmin(r0.x, gmin(r0.w, r1.z)), gmin(r0.y, gmin(r1.x, r1.w)),
                                          gmin(r0.z, gmin(r1.y, r2.x)), 0.0f);
            const float4 hi = make_float4(gmax(r0.x, gmax(r0.w, r1.z)), gmax(r0.y, gmax(r1.x, r1.w)),
                                          gmax(r0.z, gmax(r1.y, r2.x)), 0.0f);
            float nv;
            in_box = box(lo, hi, nv);
        }
        if(ls.tri && in_box)
            if(const int r = tri_test<ANY>(ls.id, make_float4(r0.x, r0.y, r0.z, r0.w), make_float4(r1.x, r1.y, r1.z, r1.w),
                                           make_float4(r2.x, r2.y, r2.z, r2.w)))
                return r;
        if(ls.parked) park();   // a triangle waiting in cur is parked next
        return 0;
    }

    // Leaf phase: the parked triangle, else the BLAS entry or triangle the
    // walk stands at.  Returns 0, or 2 (ANY only) when a triangle occludes
    // the ray.  Every lane's record - a triangle's TriRec (plus the next 16
    // bytes) or an instance's InstTrav - is read by the same four loads before
    // the kinds branch apart, so a wave with lanes of each kind waits for
    // memory once per leaf phase.
    template<bool ANY, bool COUNT>
    PTG_D int leaf_step(const DevScene& sc, Counters& cnt)
    {
        const LeafSel ls = leaf_select<ANY>(sc);
        if(ls.inst_leaf) PTG_CHECK(sc, ls.id < sc.inst_count, kDebugInst);
        if(!ls.inst_leaf) PTG_CHECK(sc, tri_base + ls.id < sc.tri_count, kDebugTri);   // read even when culled
        // every leaf lane reads its record, also a triangle whose deferred
        // near test failed (its rows then go unused): the record's address is
        // valid either way, the wave issues the same four loads, and the rows
        // need no zeroing or branch around the loads
        const v4f r0 = ls.p[0], r1 = ls.p[1], r2 = ls.p[2], r3 = ls.p[3];
        return leaf_finish<ANY, COUNT>(sc, cnt, ls, r0, r1, r2, r3);
    }

    // One step of either phase (the per-lane walks: the megakernel and the
    // per-ray entry points).  Returns 0 while the walk goes on, 1 when it
    // has ended, 2 (ANY only) when an occluder was found.
    template<bool ANY, bool COUNT>
    PTG_D int step(const DevScene& sc, Counters& cnt)
    {
        if(wants_leaf()) return leaf_step<ANY, COUNT>(sc, cnt);
        return node_step<COUNT>(sc, cnt);
    }
};

using Walker = BlockWalker<RegCold, PrivStack>;

// A whole query on one lane.  Returns whether the ray hit (ANY: occluded).
// `root` is the TLAS's root block (tlas_of), `unused` keeps the reference
// layout's (count, offset) call shape.
template<bool ANY, bool COUNT>
PTG_D bool trace(const DevScene& sc, uint32_t root, uint32_t /*unused*/, f3 o, f3 d, float tmin, float tmax, Hit& best,
                 Counters& cnt)
{
    if(COUNT) cnt.queries++;
    Walker w;
    w.init(root, o, d, tmin, tmax);
    int r;
    while((r = w.template step<ANY, COUNT>(sc, cnt)) == 0) {}
    best = w.result();
    return ANY ? r == 2 : best.thit >= 0.0f;
}

// ---- the same hot path over the reference's own arrays --------------------
// RefScene holds the nine borrowed pointers of path_trace_pixel
// (path_tracer.hh:637-654) in the reference layout (bvh.hh, mesh.hh,
// scene.hh): nodes 24 B, 8 link orders of 8 B per node, indices, 16-byte
// float3 positions/normals, float4 albedo/material, 160-byte instances and
// subframes.  trace() over a RefScene walks those arrays exactly as
// ray_query_proceed does (ray_query.hh:184-278) - no repacking - so a kernel
// can call path_trace_pixel on the arrays the reference's scene holds
// (include/ptg_device.h).  The frame renderer uses DevScene's repacked records.
struct RefScene {
    const uint8_t* subframes;        // subframe[]          (160 B)
    const uint8_t* instances;        // tlas_instance[]     (160 B)
    const float* nodes;              // bvh_node[]          (24 B)
    const uint2* links;              // bvh_link[], 8 orders per node
    const uint32_t* indices;
    const float* pos;                // float3[] (16 B stride)
    const float* normal;
    const float* albedo;             // float4[]
    const float* material;
    const float2* polygon;           // always null: the camera evaluates the aperture polygon itself
    uint32_t width, height, max_bounces, student_id, blur_step;
};

// ray_query_context (ray_query.hh:52-60)
struct RefLevel {
    uint32_t count, offset, link_offset, node;
    f3 org, inv;
};

// ray_query_traverse (ray_query.hh:184-223): next leaf payload, or 0xFFFFFFFF
PTG_D uint32_t ref_traverse(const RefScene& sc, RefLevel& c, float tmin, float tmax, Counters& cnt, bool count)
{
    while(c.node < c.count)
    {
        const float* n = sc.nodes + size_t(c.offset + c.node) * 6;
        const uint2 l = sc.links[c.link_offset + c.node];
        if(count) cnt.visits++;
        if(slab_hit(c.org, c.inv, tmin, tmax, n[0], n[1], n[2], n[3], n[4], n[5]))
        {
            const uint32_t accept = l.x & 0x7FFFFFFFu;
            if(accept != l.x) { c.node = l.y; return accept; }
            c.node = accept;
        }
        else c.node = l.y;
    }
    return 0xFFFFFFFFu;
}

PTG_D f3 ref_f3(const float* base, uint32_t i)
{
    const float4 v = reinterpret_cast<const float4*>(base)[i];
    return V3(v.x, v.y, v.z);
}

// ray_query_initialize + the proceed/confirm loop of trace_ray (ANY = false,
// path_tracer.hh:342-349) or the single proceed of trace_shadow_ray (ANY =
// true, :415-427), over the reference arrays.
template<bool ANY, bool COUNT>
PTG_D bool trace(const RefScene& sc, uint32_t tlas_count, uint32_t tlas_offset, f3 o, f3 d, float tmin, float tmax,
                 Hit& best, Counters& cnt)
{
    if(COUNT) cnt.queries++;
    RefLevel tl{tlas_count, tlas_offset, tlas_offset * 8 + octant(d) * tlas_count, 0, o,
                V3(rcp_or_big(d.x), rcp_or_big(d.y), rcp_or_big(d.z))};
    RefLevel bl{0, 0, 0, 0, V3(0, 0, 0), V3(0, 0, 0)};
    int axis = -1;
    f3 S = V3(0, 0, 0);
    uint32_t inst = 0xFFFFFFFFu, ioff = 0, bv = 0;
    best.thit = -1.0f;
    best.bx = best.by = best.bz = 0.0f;
    best.instance_id = 0xFFFFFFFFu;
    best.primitive_id = 0;
    best.back_face = false;
    for(;;)
    {
        const uint32_t leaf = ref_traverse(sc, axis < 0 ? tl : bl, tmin, tmax, cnt, COUNT);
        if(leaf == 0xFFFFFFFFu)
        {
            if(axis < 0) return ANY ? false : best.thit >= 0.0f;
            axis = -1;
            continue;
        }
        if(axis < 0)
        {   // ray_query_enter_blas (ray_query.hh:153-182)
            if(COUNT) cnt.blas_entries++;
            const uint8_t* in = sc.instances + size_t(leaf) * 160;
            const uint32_t* h = reinterpret_cast<const uint32_t*>(in);
            const float* M = reinterpret_cast<const float*>(in + 96);      // inv_transform rows
            bl.count = h[0];
            bl.offset = h[1];
            ioff = h[4];
            bv = h[5];
            inst = leaf;
            bl.org = V3(M[0] * o.x + M[4] * o.y + M[8] * o.z + M[12] * 1.0f,
                        M[1] * o.x + M[5] * o.y + M[9] * o.z + M[13] * 1.0f,
                        M[2] * o.x + M[6] * o.y + M[10] * o.z + M[14] * 1.0f);
            const f3 bd = V3(M[0] * d.x + M[4] * d.y + M[8] * d.z, M[1] * d.x + M[5] * d.y + M[9] * d.z,
                             M[2] * d.x + M[6] * d.y + M[10] * d.z);
            bl.inv = V3(rcp_or_big(bd.x), rcp_or_big(bd.y), rcp_or_big(bd.z));
            bl.link_offset = bl.offset * 8 + octant(bd) * bl.count;
            bl.node = 0;
            tri_preprocess(bd, axis, S);
            continue;
        }
        // ray_query_test_triangle (ray_query.hh:225-246)
        if(COUNT) cnt.tri_tests++;
        const uint32_t* tri = sc.indices + ioff + leaf * 3;
        float u, v, t;
        bool back;
        if(tri_accept(bl.org, axis, S, ref_f3(sc.pos, bv + tri[0]), ref_f3(sc.pos, bv + tri[1]), ref_f3(sc.pos, bv + tri[2]),
                      tmin, tmax, u, v, t, back))
        {
            if(ANY) return true;
            // ray_query_confirm (ray_query.hh:280-290)
            best.bx = u;
            best.by = v;
            best.bz = 1.0f - u - v;
            best.thit = t;
            best.instance_id = inst;
            best.primitive_id = leaf;
            best.back_face = back;
            tmax = t;
        }
    }
}

// Where the shading of a hit finds its instance: the transform's rotation
// rows (extract_m4m3) and the mesh's index / vertex offsets (path_tracer.hh:369-371).
PTG_D void shade_instance(const DevScene& sc, uint32_t id, m3& rot, uint32_t& ioff, uint32_t& bv)
{
    const float4* sp = reinterpret_cast<const float4*>(sc.inst_shade + id);
    const float4 s0 = sp[0], s1 = sp[1], s2 = sp[2];
    rot = m3{{V3(s0.x, s0.y, s0.z), V3(s0.w, s1.x, s1.y), V3(s1.z, s1.w, s2.x)}};
    ioff = __float_as_uint(s2.y);
    bv = __float_as_uint(s2.z);
}
PTG_D void shade_instance(const RefScene& sc, uint32_t id, m3& rot, uint32_t& ioff, uint32_t& bv)
{
    const uint8_t* in = sc.instances + size_t(id) * 160;
    const float* T = reinterpret_cast<const float*>(in + 32);            // transform rows
    rot = m3{{V3(T[0], T[1], T[2]), V3(T[4], T[5], T[6]), V3(T[8], T[9], T[10])}};
    ioff = reinterpret_cast<const uint32_t*>(in)[4];
    bv = reinterpret_cast<const uint32_t*>(in)[5];
}

struct HitInfo {
    float thit;
    f3 pos;
    m3 tbn;
    f3 albedo;
    float roughness, metallic, emission, transmission, eta, nee_pdf;
};

struct Light {
    f3 dir, color;
    float cos;
};

PTG_D f3 ld3(const float* base, uint32_t i)
{
    const float4 v = reinterpret_cast<const float4*>(base)[i];
    return V3(v.x, v.y, v.z);
}
PTG_D float4 ld4(const float* base, uint32_t i) { return reinterpret_cast<const float4*>(base)[i]; }

// A hit triangle's vertex attributes (path_tracer.hh:373-392): normals,
// albedos, materials of vertices indices[ioff + 3 prim + k] + bv.  The device
// scene reads them from the triangle's TriShade line (the same values,
// gathered once per mesh by k_pack_tris); the reference-layout scene gathers
// them through the indices.
struct TriAttrs {
    f3 n[3];
    float4 a[3], m[3];
};
PTG_D TriAttrs tri_attrs_at(const DevScene& sc, uint32_t tri)
{
    const float4* q = reinterpret_cast<const float4*>(sc.tri_shade + tri);
    float f[32];
#pragma unroll
    for(int r = 0; r < 8; ++r)
    {
        const float4 v = q[r];
        f[4 * r] = v.x;
        f[4 * r + 1] = v.y;
        f[4 * r + 2] = v.z;
        f[4 * r + 3] = v.w;
    }
    TriAttrs t;
#pragma unroll
    for(int k = 0; k < 3; ++k)
    {
        const float* g = f + 10 * k;
        t.n[k] = V3(g[0], g[1], g[2]);
        t.a[k] = make_float4(g[3], g[4], g[5], 0.0f);
        t.m[k] = make_float4(g[6], g[7], g[8], g[9]);
    }
    return t;
}
// KIND 1 (the wavefront's surface pass): `prim` is the walk's mesh-global
// triangle (LdsCold::kGlobalTri), so the attribute line's address does not
// wait for the instance record
template<int KIND> PTG_D TriAttrs tri_attrs(const DevScene& sc, uint32_t ioff, uint32_t, uint32_t prim)
{
    return tri_attrs_at(sc, KIND == 1 ? prim : ioff / 3u + prim);
}
template<int KIND> PTG_D TriAttrs tri_attrs(const RefScene& sc, uint32_t ioff, uint32_t bv, uint32_t prim)
{
    const uint32_t tri = ioff + prim * 3;
    const uint32_t i[3] = {sc.indices[tri] + bv, sc.indices[tri + 1] + bv, sc.indices[tri + 2] + bv};
    TriAttrs t;
#pragma unroll
    for(int k = 0; k < 3; ++k)
    {
        t.n[k] = ld3(sc.normal, i[k]);
        t.a[k] = ld4(sc.albedo, i[k]);
        t.m[k] = ld4(sc.material, i[k]);
    }
    return t;
}

// The shading half of trace_ray (path_tracer.hh:351-411): turn the closest
// hit of the ray (origin, dir) into a hit_info.
// KIND: 0 = either, 1 = the caller knows the ray hit, 2 = it knows it missed
// (lets the wavefront kernels compile only the branch they run).
template<bool COUNT, int KIND = 0, class SC>
PTG_D HitInfo hit_info(const SC& sc, const Light& L, f3 origin, f3 dir, const Hit& h, Counters& cnt)
{
    HitInfo hi;
    hi.thit = h.thit;
    hi.nee_pdf = 0;
    if(KIND == 2 || (KIND == 0 && hi.thit < 0))
    {
        const float visible = dot(L.dir, dir) > L.cos ? 1.0f : 0.0f;
        hi.nee_pdf = visible / (2.0f * PI_F * (1.0f - L.cos));
        const float w = hi.nee_pdf == 0.0f ? 1.0f : hi.nee_pdf;
        hi.albedo = V3(0.0f, 0.0f, 0.0f) + (visible * L.color) * w;
        hi.emission = 1.0f;
        hi.pos = V3(0, 0, 0);
        hi.tbn = m3{{V3(0, 0, 0), V3(0, 0, 0), V3(0, 0, 0)}};
        hi.roughness = hi.metallic = hi.transmission = hi.eta = 0.0f;
        return hi;
    }
    if(COUNT) cnt.shades++;
    hi.pos = origin + dir * h.thit;
    m3 rot;
    uint32_t ioff, bv;
    shade_instance(sc, h.instance_id, rot, ioff, bv);
    const TriAttrs ta = tri_attrs<KIND>(sc, ioff, bv, h.primitive_id);
    const f3 n0 = ta.n[0], n1 = ta.n[1], n2 = ta.n[2];
    const float4 a0 = ta.a[0], a1 = ta.a[1], a2 = ta.a[2];
    const float4 m0 = ta.m[0], m1 = ta.m[1], m2 = ta.m[2];
    const float bx = h.bx, by = h.by, bz = h.bz;
    hi.albedo = V3(a0.x * bx + a1.x * by + a2.x * bz, a0.y * bx + a1.y * by + a2.y * bz, a0.z * bx + a1.z * by + a2.z * bz);
    const float mx = m0.x * bx + m1.x * by + m2.x * bz;
    hi.metallic = m0.y * bx + m1.y * by + m2.y * bz;
    hi.transmission = m0.z * bx + m1.z * by + m2.z * bz;
    hi.emission = m0.w * bx + m1.w * by + m2.w * bz;
    f3 n = (n0 * bx + n1 * by) + n2 * bz;
    n = normalize(mul_m3v3(rot, n));
    const float ior = 1.5f;
    if(h.back_face) { hi.eta = ior; n = -n; }
    else hi.eta = 1.0f / ior;
    hi.tbn = tangent_space(n);
    hi.roughness = mx * mx;
    return hi;
}

// trace_ray (path_tracer.hh:340-412)
template<bool COUNT, class SC>
PTG_D HitInfo trace_ray(const SC& sc, uint32_t tc, uint32_t to, const Light& L, f3 origin, f3 dir, float tmin,
                        Counters& cnt)
{
    Hit h;
    trace<false, COUNT>(sc, tc, to, origin, dir, tmin, 1e9f, h, cnt);
    return hit_info<COUNT, 0>(sc, L, origin, dir, h, cnt);
}

// ---- samplers (path_tracer.hh:12-83) ----
PTG_D float inv_erf(float x)                                          // math.hh:455-463
{
    const float ln1x2 = (float)dlog((double)(1 - x * x));
    const float a = 0.147f;
    const float p = 2.0f / (PI_F * a);
    const float k = p + ln1x2 * 0.5f;
    const float k2 = k * k;
    const double inner = dsqrt((double)(k2 - ln1x2 * (1.0f / a)));
    return (float)((double)signf(x) * dsqrt(inner - (double)k));
}
PTG_D f2 gaussian_disk(f2 u, float sigma)                              // :19-25 with sample_gaussian :12-17
{
    float r = fsqrt(u.x);
    const float theta = 2.0f * PI_F * u.y;
    float kk = r * 2.0f - 1.0f;
    kk = clampf(kk, -(1.0f - 1e-6f), 1.0f - 1e-6f);
    r = sigma * 1.41421356f * inv_erf(kk);
    return f2{r * fcos(theta), r * fsin(theta)};
}
PTG_D f3 cosine_hemisphere(f2 u)                                       // :27-33
{
    const float r = fsqrt(u.x);
    const float theta = 2.0f * PI_F * u.y;
    const f2 d{r * fcos(theta), r * fsin(theta)};
    return V3(d.x, d.y, fsqrt(gmax(0.0f, 1.0f - (d.x * d.x + d.y * d.y))));
}
PTG_D float cosine_pdf(f3 d) { return gmax(d.z * (1.0f / PI_F), 0.0f); }   // :35-38
PTG_D f3 sample_cone(f3 dir, float cos_min, f2 u)                      // :40-48
{
    const float ct = mixf(1.0f, cos_min, u.x);
    const float st = fsqrt(1.0f - ct * ct);
    const float phi = u.y * 2.0f * PI_F;
    return mul_m3v3(tangent_space(dir), V3(fcos(phi) * st, fsin(phi) * st, ct));
}
// Vertex k of the aperture polygon: angle side_radians * k + angle, as
// regular_polygon forms it for k = side and k = side + 1 (side + 1.0f is the
// float k exactly); (sin, cos) in double, rounded to float.
PTG_D f2 polygon_vertex(float angle, uint32_t sides, float k)
{
    const float side_radians = (2.0f * PI_F) / (float)sides;
    const float a = side_radians * k + angle;
    return f2{fsin(a), fcos(a)};
}
// table: the polygon_vertex values of this subframe (k = 0 .. sides + 1), or null
PTG_D f2 regular_polygon(f2 u, float angle, uint32_t sides, const float2* table = nullptr)   // :50-62
{
    const float side = (float)floor((double)(u.x * (float)sides));
    u.x *= (float)sides;
    u.x = (float)((double)u.x - floor((double)u.x));
    f2 b, c;
    if(table)
    {   // side is an integer in [0, sides] (u.x may round to 1.0)
        const float2 tb = table[(uint32_t)side], tc = table[(uint32_t)side + 1u];
        b = f2{tb.x, tb.y};
        c = f2{tc.x, tc.y};
    }
    else
    {
        b = polygon_vertex(angle, sides, side);
        c = polygon_vertex(angle, sides, side + 1.0f);
    }
    if(u.x + u.y > 1.0f) { u.x = 1.0f - u.x; u.y = 1.0f - u.y; }
    return f2{b.x * u.x + c.x * u.y, b.y * u.x + c.y * u.y};
}
template<class MP> PTG_D f3 ggx_vndf(f3 view, float roughness, f2 u, MP& mp)   // :67-83
{
    if(roughness < 1e-3f) return V3(0, 0, 1);
    const f3 v = normalize(V3(roughness * view.x, roughness * view.y, view.z));
    const float phi = 2.0f * PI_F * u.x;
    const float z = (float)fma((double)(1.0f - u.y), (double)(1.0f + v.z), (double)(-v.z));
    const float sin_theta = fsqrt(clampf(1.0f - z * z, 0.0f, 1.0f));
    const float x = times_cos(sin_theta, (double)phi, mp);
    const float y = times_sin(sin_theta, (double)phi, mp);
    const f3 h = V3(x, y, z) + v;
    return normalize(V3(roughness * h.x, roughness * h.y, gmax(0.0f, h.z)));
}

// ---- materials (path_tracer.hh:89-296) ----
template<class MP> PTG_D float fresnel_att(float vdh, float f0, float eta, float roughness, MP& mp)   // :89-98
{
    if(eta > 1.0f)
    {
        const float s2 = eta * eta * (1.0f - vdh * vdh);
        if(s2 >= 1.0f) return 1.0f;
        vdh = fsqrt(1.0f - s2);
    }
    return add_mul_pow(f0, gmax(1.0f - roughness, f0) - f0, (double)gmax(1.0f - vdh, 0.0f), 5.0, mp);
}
PTG_D float tr_distribution(float hdotn, float a)                            // :105-110
{
    const float a2 = a * a;
    const float denom = hdotn * hdotn * (a2 - 1.0f) + 1.0f;
    return a2 / gmax(PI_F * denom * denom, 1e-10f);
}
PTG_D float tr_masking_shadowing(float ldotn, float ldoth, float vdotn, float vdoth, float a)   // :112-123
{
    if(vdotn * vdoth < 0) return 0;
    if(ldotn * ldoth < 0) return 0;
    const double l = fabs((double)vdotn) * dsqrt((double)(ldotn * ldotn - a * a * ldotn * ldotn + a * a));
    const double v = fabs((double)ldotn) * dsqrt((double)(vdotn * vdotn - a * a * vdotn * vdotn + a * a));
    return (float)(0.5 / (l + v));
}
PTG_D float tr_masking(float vdotn, float vdoth, float a)                    // :125-129
{
    if(vdotn * vdoth < 0) return 0;
    return (float)((double)(2.0f * vdotn) / ((double)vdotn + dsqrt((double)(vdotn * vdotn * (1.0f - a * a) + a * a))));
}

struct Material {
    f3 albedo;
    float roughness, metallic, transmission, eta;
};

// bsdf_core (:131-181)
template<class MP>
PTG_D f3 bsdf_core(f3 light, f3 h, f3 view, const Material& M, float f0, float distribution, float& rpdf,
                   float& dpdf, float& tpdf, MP& mp)
{
    const float ldotn = light.z, vdotn = view.z;
    const float vdoth = dot(view, h), ldoth = dot(light, h);
    const float fresnel = fresnel_att(vdoth, f0, M.eta, 0, mp);
    const float geometry = tr_masking_shadowing(ldotn, ldoth, vdotn, vdoth, M.roughness);
    const float G1 = tr_masking(vdotn, vdoth, M.roughness);
    f3 color;
    if(light.z > 0)
    {
        const float spec = fresnel * (1.0f - M.metallic);
        color = V3((M.albedo.x * M.metallic + spec) * geometry * distribution,
                   (M.albedo.y * M.metallic + spec) * geometry * distribution,
                   (M.albedo.z * M.metallic + spec) * geometry * distribution);
        const float diffuse = (1.0f - fresnel) * (1.0f - M.metallic) * (1.0f - M.transmission) / PI_F;
        color = color + diffuse * M.albedo;
        rpdf = G1 * distribution / (4.0f * view.z);
        dpdf = cosine_pdf(light);
        tpdf = 0;
    }
    else
    {
        const float denom = M.eta * vdoth + ldoth;
        const double k = (double)M.transmission * fabs((double)(vdoth * ldoth)) * (double)(1.0f - fresnel) * 4.0 *
                         (double)geometry * (double)distribution / (double)(denom * denom);
        color = M.albedo * (float)k;
        rpdf = 0;
        dpdf = 0;
        tpdf = (float)(fabs((double)(vdoth * ldoth)) * (double)G1 * (double)distribution /
                       (fabs((double)view.z) * (double)denom * (double)denom));
    }
    return color * fabsf(ldotn);
}

template<class MP> PTG_D void lobe_probs(f3 view, const Material& M, float& f0, float& rp, float& tp, float& dp, MP& mp)
{
    float f = (1.0f - M.eta) / (1.0f + M.eta);
    f *= f;
    f0 = f;
    const float lum = dot(M.albedo, V3(0.2126f, 0.7152f, 0.0722f));
    rp = mixf(1.0f, fresnel_att(view.z, f, M.eta, M.roughness, mp), lum * (1.0f - M.metallic));
    tp = (float)((1.0 - (double)rp) * (double)M.transmission);
    dp = (float)((1.0 - (double)rp) * (double)(1.0f - M.transmission));
}

// bsdf (:184-222)
template<class MP> PTG_D f3 bsdf_eval(f3 light, f3 view, const Material& M, float& out_pdf, MP& mp)
{
    f3 h;
    if(light.z > 0) h = normalize(view + light);
    else h = signf(M.eta - 1.0f) * normalize(light + M.eta * view);
    const float distribution = tr_distribution(h.z, M.roughness);
    float f0, rp, tp, dp;
    lobe_probs(view, M, f0, rp, tp, dp, mp);
    float r, d, t;
    const f3 att = bsdf_core(light, h, view, M, f0, M.roughness < 1e-3f ? 0.0f : distribution, r, d, t, mp);
    out_pdf = r * rp + d * dp + t * tp;
    return att;
}

// sample_bsdf (:224-296)
template<class MP> PTG_D void bsdf_sample(f3 u, f3 view, const Material& M, f3& out_dir, f3& out_att, float& out_pdf, MP& mp)
{
    const f2 uxy{u.x, u.y};
    f3 h = ggx_vndf(view, M.roughness, uxy, mp);
    float f0, rp, tp, dp;
    lobe_probs(view, M, f0, rp, tp, dp, mp);
    bool diffuse = false, bad;
    if((u.z -= rp) <= 0)
    {   // reflect(-view, h) (math.hh:442-445)
        const f3 I = -view;
        out_dir = I - (2.0f * dot(h, I)) * h;
        bad = out_dir.z <= 0;
    }
    else if((u.z -= tp) <= 0)
    {   // refract(-view, h, eta) (math.hh:447-453)
        const f3 I = -view;
        const float ndoti = dot(h, I);
        const float k = 1.0f - M.eta * M.eta * (1.0f - ndoti * ndoti);
        if(k < 0.0f) out_dir = V3(0, 0, 0);
        else
        {
            const float s = (float)((double)(M.eta * ndoti) + dsqrt((double)k));
            out_dir = M.eta * I - s * h;
        }
        bad = out_dir.z >= 0;
    }
    else
    {
        out_dir = cosine_hemisphere(uxy);
        h = normalize(out_dir + view);
        diffuse = true;
        bad = out_dir.z == 0;
    }
    if(bad)
    {
        out_dir = V3(0, 0, 1);
        out_att = V3(0, 0, 0);
        out_pdf = 1;
        return;
    }
    float distribution = tr_distribution(h.z, M.roughness);
    if(M.roughness < 1e-3f) distribution = diffuse ? 0 : fabsf(4.0f * out_dir.z * view.z);
    float r, d, t;
    out_att = bsdf_core(out_dir, h, view, M, f0, distribution, r, d, t, mp);
    out_pdf = r * rp + t * tp;
    if(M.roughness < 1e-3f && !diffuse) out_pdf = -out_pdf;
    else out_pdf += d * dp;
}

// ray_sphere_intersection (math.hh:404-417)
PTG_D bool ray_sphere(f3 o, f3 d, f3 c, float radius, float& tmin, float& tmax)
{
    const f3 oc = o - c;
    const float b = dot(oc, d);
    const float cc = dot(oc, oc) - radius * radius;
    float disc = b * b - cc;
    if(disc < 0) return false;
    disc = fsqrt(disc);
    tmin = -b - disc;
    tmax = -b + disc;
    return true;
}

constexpr float RAY_R = 5.8e-6f, RAY_G = 13.6e-6f, RAY_B = 33.1e-6f, MIE_K = 4.0e-6f;

// The prologue of nishita_atmosphere_attenuation (:456-497): whether the ray
// misses the atmosphere (attenuation 1), its primary step length, and whether
// one of its steps lies below the ground (attenuation exactly 0).  The
// reference sums the depths over every step and then returns 0 if a step lay
// below the ground; the sums are only read when none did, so the heights are
// tested first and the exp work is skipped for a shadowed ray (the same
// result; the heights are recomputed bit for bit).
struct AttenSteps {
    bool outside, blocked;
    float segment;
};
PTG_D AttenSteps attenuation_steps(float jitter, f3 pos, f3 view, float tmax)
{
    const f3 earth = V3(0, -EARTH_RADIUS, 0);
    AttenSteps a{false, false, 0.0f};
    float tmin = 0, atmax = 0;
    if(!ray_sphere(pos, view, earth, EARTH_RADIUS + ATMOSPHERE_HEIGHT, tmin, atmax))
    {
        a.outside = true;
        return a;
    }
    tmin = (float)gmax_d((double)tmin, 0.0);
    tmax = gmin(atmax, tmax < 0 ? MAX_RAY_DIST : tmax);
    a.segment = (tmax - tmin) / (float)PRIMARY_ITERATIONS;
    for(int i = 0; i < PRIMARY_ITERATIONS; ++i)
    {
        const float t = a.segment * (jitter + (float)i);
        if(length((pos + t * view) - earth) - EARTH_RADIUS < 0)
        {
            a.blocked = true;
            return a;
        }
    }
    return a;
}

// nishita_atmosphere_attenuation (:456-497)
template<class MP> PTG_D f3 atmosphere_attenuation(float jitter, f3 pos, f3 view, float tmax, MP& mp)
{
    const f3 earth = V3(0, -EARTH_RADIUS, 0);
    const AttenSteps a = attenuation_steps(jitter, pos, view, tmax);
    if(a.outside) return V3(1.0f, 1.0f, 1.0f);
    if(a.blocked) return V3(0.0f, 0.0f, 0.0f);
    const float segment = a.segment;
    float ray_depth = 0, mie_depth = 0;
    for(int i = 0; i < PRIMARY_ITERATIONS; ++i)
    {
        const float t = segment * (jitter + (float)i);
        const float height = length((pos + t * view) - earth) - EARTH_RADIUS;
        ray_depth = acc_exp(ray_depth, (double)ray_h(height), mp);
        mie_depth = acc_exp(mie_depth, (double)mie_h(height), mp);
    }
    const f3 tau = V3((RAY_R * ray_depth + MIE_K * mie_depth) * segment, (RAY_G * ray_depth + MIE_K * mie_depth) * segment,
                      (RAY_B * ray_depth + MIE_K * mie_depth) * segment);
    return V3(fexp(-tau.x), fexp(-tau.y), fexp(-tau.z));
}

// nishita_atmosphere_scattering (:499-588)
template<class MP>
PTG_D void atmosphere_scattering(u4& seed, const Light& L, f3 pos, f3 view, float tmax, f3& attenuation, f3& in_scatter,
                                 MP& mp)
{
    const f3 earth = V3(0, -EARTH_RADIUS, 0);
    attenuation = V3(1.0f, 1.0f, 1.0f);
    in_scatter = V3(0.0f, 0.0f, 0.0f);
    if(tmax > 0 && tmax < 1e3f) return;
    float tmin = 0, atmax = 0;
    if(!ray_sphere(pos, view, earth, EARTH_RADIUS + ATMOSPHERE_HEIGHT, tmin, atmax)) return;
    tmin = (float)gmax_d((double)tmin, 0.0);
    tmax = gmin(atmax, tmax < 0 ? MAX_RAY_DIST : tmax);
    const float segment = (tmax - tmin) / (float)PRIMARY_ITERATIONS;
    const f4 jitter = uniform4(seed);
    const float mu = dot(view, L.dir);
    const float rayleigh_phase = 3.0f / (16.0f * PI_F) * (1.0f + mu * mu);
    const float g = MIE_ANISOTROPY;
    const float mie_phase = div_mul_pow((double)(3.0f / (8.0f * PI_F) * (1.0f - g * g) * (1.0f + mu * mu)),
                                        (double)(2.0f + g * g), (double)(1.0f + g * g - 2.0f * g * mu), 1.5, mp);
    float ray_depth = 0, mie_depth = 0;
    f3 ray_sum = V3(0, 0, 0), mie_sum = V3(0, 0, 0);
    for(int i = 0; i < PRIMARY_ITERATIONS; ++i)
    {
        const float t = segment * (jitter.x + (float)i);
        const f3 p = pos + t * view;
        ray_sphere(p, L.dir, earth, EARTH_RADIUS + ATMOSPHERE_HEIGHT, tmin, tmax);   // keeps old values on a miss
        const float light_segment = (tmax - tmin) / (float)SECONDARY_ITERATIONS;
        float lray = 0, lmie = 0;
        bool shadowed = false;   // lray / lmie are read only if not (heights tested first, as above)
        for(int j = 0; j < SECONDARY_ITERATIONS; ++j)
        {
            const float tt = light_segment * (jitter.y + (float)j);
            if(length((p + tt * L.dir) - earth) - EARTH_RADIUS < 0) shadowed = true;
        }
        if(!shadowed)
            for(int j = 0; j < SECONDARY_ITERATIONS; ++j)
            {
                const float tt = light_segment * (jitter.y + (float)j);
                const float height = length((p + tt * L.dir) - earth) - EARTH_RADIUS;
                lray = acc_exp(lray, (double)ray_h(height), mp);
                lmie = acc_exp(lmie, (double)mie_h(height), mp);
            }
        const float height = gmax(length(p - earth) - EARTH_RADIUS, 0.0f);
        const float ray_density = exp_times((double)ray_h(height), segment, mp);
        const float mie_density = exp_times((double)mie_h(height), segment, mp);
        ray_depth += ray_density;
        mie_depth += mie_density;
        const float kr = lray * light_segment + ray_depth, km = lmie * light_segment + mie_depth;
        f3 local = V3(0.0f, 0.0f, 0.0f);
        if(!shadowed)
            local = V3(fexp(-(RAY_R * kr + MIE_K * km)), fexp(-(RAY_G * kr + MIE_K * km)),
                       fexp(-(RAY_B * kr + MIE_K * km)));
        ray_sum = ray_sum + local * ray_density;
        mie_sum = mie_sum + local * mie_density;
    }
    attenuation = V3(fexp(-(RAY_R * ray_depth + MIE_K * mie_depth)), fexp(-(RAY_G * ray_depth + MIE_K * mie_depth)),
                     fexp(-(RAY_B * ray_depth + MIE_K * mie_depth)));
    const f3 R = V3(RAY_R, RAY_G, RAY_B), Mk = V3(MIE_K, MIE_K, MIE_K);
    in_scatter = ((((ray_sum * R) * rayleigh_phase) + ((mie_sum * Mk) * mie_phase)) * L.color) * 4.0f;
}

// nee_branch (:594-620), split at its shadow ray so the wavefront pipeline
// can trace that ray in a separate kernel:
//   nee_prepare: the NEE random draw, the sun-cone direction, the BSDF value
//                and MIS weight; returns false when the colour is zero (the
//                reference then returns 0 without tracing);
//   nee_finish:  for an unoccluded shadow ray, the transmittance along it and
//                the MIS division.
struct NeeCandidate {
    f3 color, dir;
    float mis_pdf, jitter;
};

template<class MP>
PTG_D bool nee_prepare(u4& seed, const Light& L, const HitInfo& info, const Material& M, f3 tview, NeeCandidate& c, MP& mp)
{
    const f4 u = uniform4(seed);
    c.dir = sample_cone(L.dir, L.cos, f2{u.x, u.y});
    c.jitter = u.w;
    const float nee_pdf = 1.0f / (2.0f * PI_F * (1.0f - L.cos));
    float bsdf_pdf = 0;
    const f3 b = bsdf_eval(mul_v3m3(c.dir, info.tbn), tview, M, bsdf_pdf, mp);
    c.color = (b * nee_pdf) * L.color;
    c.mis_pdf = 1.0f;
    if(L.cos < 1.0f) c.mis_pdf = (nee_pdf * nee_pdf + bsdf_pdf * bsdf_pdf) / nee_pdf;
    return !(c.color.x == 0 && c.color.y == 0 && c.color.z == 0);
}

template<class MP> PTG_D f3 nee_finish(const NeeCandidate& c, f3 pos, MP& mp)
{
    const f3 color = c.color * atmosphere_attenuation(c.jitter, pos, c.dir, MAX_RAY_DIST, mp);
    return color / c.mis_pdf;
}

// Whether the shadow ray of a prepared NEE candidate can be left untraced:
// when one step of the sun ray's atmosphere integral lies below the ground,
// the attenuation is exactly 0 before any exp (attenuation_steps), and if
// nee_finish's value, (colour * 0) / mis_pdf, is then +0 in every component,
// it is bitwise the V3(0, 0, 0) an occluded ray gives: the next round adds
// att * (+0) either way.  Only the occlusion test is skipped; the random
// draws and every value are the reference's.
PTG_D bool nee_shadow_moot(const NeeCandidate& c, f3 pos)
{
    if(!attenuation_steps(c.jitter, pos, c.dir, MAX_RAY_DIST).blocked) return false;
    const f3 z = (c.color * V3(0.0f, 0.0f, 0.0f)) / c.mis_pdf;
    return (__float_as_uint(z.x) | __float_as_uint(z.y) | __float_as_uint(z.z)) == 0u;
}

// Whether the shadow ray of a prepared NEE candidate can be left untraced
// because the path's throughput is exactly zero (a BSDF sample of zero
// weight made it so: 10-13% of all bounces on frames 0, 450 and 1400).  The
// reference adds contrib + att * nee_branch(...) (path_tracer.hh:705; the
// wavefront adds it at the start of the next round, with this same att and
// contrib).  With every component of att +-0 and the unoccluded value
// (colour * A) / mis_pdf finite - colour finite, mis_pdf finite and
// positive, and the atmosphere's transmittance A in [+0, 1]
// (nishita_atmosphere_attenuation: exp of a non-positive float, 1 outside
// the atmosphere, 0 below the ground) - both att * nee (unoccluded) and
// att * (+0) (occluded) are zeros; x + (+-0) == x bitwise for every x but
// -0, where the sum takes the term's sign: att's sign XOR the colour's when
// unoccluded, att's alone when occluded.  So a -0 component of contrib needs
// a colour component without its sign bit.  NaN throughput never qualifies.
PTG_D bool nee_term_moot(f3 att, f3 contrib, const NeeCandidate& c)
{
    const uint32_t az = (__float_as_uint(att.x) | __float_as_uint(att.y) | __float_as_uint(att.z)) & 0x7FFFFFFFu;
    if(az != 0u) return false;
    if(!finite3(c.color) || !(c.mis_pdf > 0.0f) || !__builtin_isfinite(c.mis_pdf)) return false;
    // (colour * A) / mis_pdf with A in [+0, 1] is at most colour / mis_pdf in
    // magnitude (rounding is monotone): finite when that is (a colour near
    // FLT_MAX from ptg_upload_frame could otherwise overflow to inf)
    if(!finite3(c.color / c.mis_pdf)) return false;
    const bool neg0x = __float_as_uint(contrib.x) == 0x80000000u && (__float_as_uint(c.color.x) >> 31);
    const bool neg0y = __float_as_uint(contrib.y) == 0x80000000u && (__float_as_uint(c.color.y) >> 31);
    const bool neg0z = __float_as_uint(contrib.z) == 0x80000000u && (__float_as_uint(c.color.z) >> 31);
    return !(neg0x || neg0y || neg0z);
}

// Whether a path whose throughput is exactly zero can be retired at its
// last bounce, with its contribution as it stands, instead of tracing that
// bounce's ray (the reference's last loop iteration, path_tracer.hh:697-738,
// with no NEE ray pending: nee_term_moot held).  What that iteration would
// still add is contrib + att * (+0) (the untraced NEE term) and contrib +
// (att * batt) * X / mis_pdf (bounce_tail), X = insc + (aatt * albedo) *
// emission.  With att +-0, batt finite, X finite (a hit: finite vertex data,
// `attrs_finite`; a miss: the sun-disk term and the atmosphere integrals,
// see bounce_tail) and mis_pdf neither 0 nor NaN for the hit and for both
// miss cases (nee_pdf 0 or the sun disk's, hit_info), both terms are +-0;
// and x + (+-0) == x bitwise for every x but -0, which contrib must not hold.
// The sky's terms of a retiring path - the sun-disk albedo (visible * colour)
// * w with w the disk's pdf 1 / (2 pi (1 - cos)), and the in-scatter, the
// colour times the atmosphere's bounded integrals (at most ~1e3 over the 8 x 4
// steps, nishita_atmosphere_scattering) - are finite when the colour is finite
// and its magnitude times max(w, 1) stays below 2^100 (2^28 of headroom).  The
// zero-throughput shortcuts need X finite; a light from ptg_upload_frame is
// not validated, so a NaN, infinite or huge colour, or a degenerate cone,
// takes the full computation.
PTG_D bool sky_terms_finite(const Light& L)
{
    const float sun = 1.0f / (2.0f * PI_F * (1.0f - L.cos));
    if(!finite3(L.color) || !__builtin_isfinite(sun)) return false;
    const float m = gmax(fabsf(L.color.x), gmax(fabsf(L.color.y), fabsf(L.color.z))) * gmax(fabsf(sun), 1.0f);
    return m < 0x1p100f;
}

PTG_D bool last_bounce_moot(f3 att, f3 batt, float bpdf, f3 contrib, const Light& L)
{
    const uint32_t az = (__float_as_uint(att.x) | __float_as_uint(att.y) | __float_as_uint(att.z)) & 0x7FFFFFFFu;
    if(az != 0u || !finite3(batt) || !sky_terms_finite(L)) return false;
    if(__float_as_uint(contrib.x) == 0x80000000u || __float_as_uint(contrib.y) == 0x80000000u ||
       __float_as_uint(contrib.z) == 0x80000000u)
        return false;
    if(bpdf < 0) return true;   // mis_pdf = -bpdf: nonzero, not NaN
    const float sun = 1.0f / (2.0f * PI_F * (1.0f - L.cos));   // hit_info's nee_pdf of a visible sun disk
    const float m0 = (0.0f * 0.0f + bpdf * bpdf) / bpdf, m1 = (sun * sun + bpdf * bpdf) / bpdf;
    return m0 != 0.0f && m0 == m0 && m1 != 0.0f && m1 == m1;
}

template<bool COUNT, class SC>
PTG_D f3 nee_branch(const SC& sc, uint32_t tc, uint32_t to, u4& seed, const Light& L, const HitInfo& info,
                    const Material& M, f3 tview, Counters& cnt, MathExact& mx)
{
    NeeCandidate c;
    if(!nee_prepare(seed, L, info, M, tview, c, mx)) return V3(0, 0, 0);
    Hit unused;
    if(trace<true, COUNT>(sc, tc, to, info.pos, c.dir, MIN_RAY_DIST, MAX_RAY_DIST, unused, cnt)) return V3(0, 0, 0);
    return nee_finish(c, info.pos, mx);
}

PTG_D float rd_f(const uint8_t* p, uint32_t off) { return *reinterpret_cast<const float*>(p + off); }
PTG_D uint32_t rd_u(const uint8_t* p, uint32_t off) { return *reinterpret_cast<const uint32_t*>(p + off); }
PTG_D f3 rd_f3(const uint8_t* p, uint32_t off)
{
    const float4 v = *reinterpret_cast<const float4*>(p + off);
    return V3(v.x, v.y, v.z);
}

// subframes[sample_index / SAMPLES_PER_MOTION_BLUR_STEP] (path_tracer.hh:655-657)
template<class SC>
PTG_D const uint8_t* subframe_of(const SC& sc, int32_t sample_index)
{
    const uint32_t sub = sample_index < 0 ? 0u : (uint32_t)sample_index / sc.blur_step;
    return sc.subframes + size_t(sub) * SF_STRIDE;
}
PTG_D Light light_of(const uint8_t* sf)
{
    Light L;
    L.dir = rd_f3(sf, SF_LIGHT);
    L.color = rd_f3(sf, SF_LIGHT + 16);
    L.cos = rd_f(sf, SF_LIGHT + 32);
    return L;
}

// Seed initialisation, film jitter and get_camera_ray (path_tracer.hh:659-671, :429-450).
template<class SC>
PTG_D void camera_ray(const SC& sc, const uint8_t* sf, uint32_t px, uint32_t py, int32_t sample_index, u4& seed,
                      f3& ray_o, f3& ray_dir)
{
    seed = u4{px, py, (uint32_t)sample_index, sc.student_id};
    pcg4d(seed);
    const f4 u = uniform4(seed);
    f2 film = gaussian_disk(f2{u.x, u.y}, 0.4f);
    film.x = film.x + 0.5f;
    film.y = film.y + 0.5f;
    const uint8_t* cam = sf + SF_CAM;
    float uvx = ((float)px + film.x) / (float)sc.width * 2.0f - 1.0f;
    float uvy = ((float)py + film.y) / (float)sc.height * 2.0f - 1.0f;
    uvx *= rd_f(cam, 64);
    uvy = -uvy;
    f2 ap{0, 0};
    const int32_t polygon = (int32_t)rd_u(cam, 80);
    if(polygon > 3)
    {
        const uint32_t sub = (uint32_t)(sf - sc.subframes) / SF_STRIDE;
        const float2* table = (sc.polygon && (uint32_t)polygon <= kPolyMaxSides) ? sc.polygon + size_t(sub) * kPolyStride
                                                                                 : nullptr;
        const f2 p = regular_polygon(f2{u.z, u.w}, rd_f(cam, 76), (uint32_t)polygon, table);
        const float rad = rd_f(cam, 84);
        ap = f2{p.x * rad, p.y * rad};
    }
    const f3 origin = V3(ap.x, ap.y, 0.0f);
    const float ifl = rd_f(cam, 68), fd = rd_f(cam, 72);
    f3 d = V3(uvx * ifl * fd, uvy * ifl * fd, -1.0f * fd);
    d = normalize(d - origin);
    const m3 ori{{rd_f3(cam, 0), rd_f3(cam, 16), rd_f3(cam, 32)}};
    ray_dir = mul_m3v3(ori, d);
    ray_o = mul_m3v3(ori, origin) + rd_f3(cam, 48);
}

// The bounce-loop head (path_tracer.hh:699-702): tangent-space view vector.
PTG_D f3 tangent_view(f3 ray_dir, const HitInfo& info)
{
    f3 view = mul_v3m3(-ray_dir, info.tbn);
    if(view.z < 1e-7f) view.z = gmax(view.z, 1e-7f);
    return normalize(view);
}

// After tracing bounce ray `ray_dir` from `ray_o` (path_tracer.hh:722-737):
// MIS, throughput, atmosphere, contribution, path-space regularisation.
// NEED_REG = false: the caller retires the path after this, so the
// regularised roughness is never read (the certified sky pass would otherwise
// spend a pow and its certificate on a dead value).
template<class MP, bool NEED_REG = true>
PTG_D void bounce_tail(u4& seed, const Light& L, f3 ray_o, f3 ray_dir, HitInfo& info, f3 batt, float bpdf,
                       f3& attenuation, f3& contribution, float& regularization, MP& mp)
{
    const float mis_pdf = bpdf < 0 ? -bpdf : (info.nee_pdf * info.nee_pdf + bpdf * bpdf) / bpdf;
    attenuation = attenuation * batt;
#ifndef PTG_ZERO_ATT_SKY
#define PTG_ZERO_ATT_SKY 1
#endif
    if constexpr(!NEED_REG && PTG_ZERO_ATT_SKY)
    {   // The path retires here (the sky pass: its ray left the scene).  With
        // the throughput exactly +-0 in every component the term is
        // att * X / mis_pdf with X = insc + (aatt * albedo) * emission finite
        // and without a sign bit: the in-scatter and the transmittance are
        // sums and products of exp values (nishita_atmosphere_scattering,
        // path_tracer.hh:499-588: a shadowed step's infinite optical depth
        // only feeds an attenuation that is then set to 0), the albedo is
        // the sun-disk term (visible * colour) * w >= +0 for a colour without
        // sign bits, the emission 1.  So att * X is att * (+0) bit for bit
        // (+-0 with att's signs), and with mis_pdf finite and nonzero the
        // contribution takes the same bits without the integrals; their one
        // random draw only feeds this retired path.
        const uint32_t az = (__float_as_uint(attenuation.x) | __float_as_uint(attenuation.y) |
                             __float_as_uint(attenuation.z)) & 0x7FFFFFFFu;
        const uint32_t colour_signs = (__float_as_uint(L.color.x) | __float_as_uint(L.color.y) |
                                       __float_as_uint(L.color.z)) >> 31;
        if(az == 0u && colour_signs == 0u && __builtin_isfinite(mis_pdf) && mis_pdf != 0.0f && sky_terms_finite(L))
        {
            contribution = contribution + (attenuation * V3(0.0f, 0.0f, 0.0f)) / mis_pdf;
            return;
        }
    }
    f3 aatt, insc;
    atmosphere_scattering(seed, L, ray_o, ray_dir, info.thit, aatt, insc, mp);
    const f3 term = attenuation * (insc + (aatt * info.albedo) * info.emission);
    contribution = contribution + term / mis_pdf;
    attenuation = attenuation * (aatt / fabsf(bpdf));
    if(!NEED_REG) return;
    if(bpdf > 0.0f)
        regularization = times_one_minus_div_pow(regularization, (double)REGULARIZATION_GAMMA, (double)bpdf, 0.25, mp);
    info.roughness = 1.0f - (1.0f - info.roughness) * regularization;
}

// A subframe's TLAS handle in the form the scene's trace() takes: the root
// block of its packed TLAS (DevScene), or the reference's (node_count,
// node_offset) pair (RefScene, scene.hh:26-34).
PTG_D void tlas_of(const DevScene& sc, const uint8_t* sf, uint32_t& a, uint32_t& b)
{
    a = sc.tlas_root[uint32_t(sf - sc.subframes) / SF_STRIDE];
    b = 0;
}
PTG_D void tlas_of(const RefScene&, const uint8_t* sf, uint32_t& a, uint32_t& b)
{
    a = rd_u(sf, SF_TLAS);
    b = rd_u(sf, SF_TLAS + 4);
}

// path_trace_pixel (path_tracer.hh:637-741) as one device function (used by
// the per-sample entry point; the frame renderer runs the same steps as a
// wavefront pipeline, csrc/device/wavefront.h).
template<bool COUNT, class SC>
PTG_D f3 path_trace_sample(const SC& sc, uint32_t px, uint32_t py, int32_t sample_index, Counters& cnt)
{
    const uint8_t* sf = subframe_of(sc, sample_index);
    uint32_t tc, to;
    tlas_of(sc, sf, tc, to);
    const Light L = light_of(sf);
    u4 seed;
    f3 ray_o, ray_dir;
    camera_ray(sc, sf, px, py, sample_index, seed, ray_o, ray_dir);

    MathExact mx;   // glibc's double library algorithms throughout
    HitInfo info = trace_ray<COUNT>(sc, tc, to, L, ray_o, ray_dir, 0.0f, cnt);
    f3 attenuation, in_scatter;
    atmosphere_scattering(seed, L, ray_o, ray_dir, info.thit, attenuation, in_scatter, mx);
    f3 contribution = V3(0, 0, 0) + (in_scatter + (attenuation * info.albedo) * info.emission);

    float regularization = 1.0f;
    for(uint32_t bounce = 0; bounce < sc.max_bounces && info.thit > 0; ++bounce)
    {
        const Material M{info.albedo, info.roughness, info.metallic, info.transmission, info.eta};
        const f3 view = tangent_view(ray_dir, info);
        contribution = contribution + attenuation * nee_branch<COUNT>(sc, tc, to, seed, L, info, M, view, cnt, mx);
        const f4 ub = uniform4(seed);
        f3 tdir, batt;
        float bpdf;
        bsdf_sample(V3(ub.x, ub.y, ub.z), view, M, tdir, batt, bpdf, mx);
        ray_dir = normalize(mul_m3v3(info.tbn, tdir));
        ray_o = info.pos;
        info = trace_ray<COUNT>(sc, tc, to, L, ray_o, ray_dir, MIN_RAY_DIST, cnt);
        bounce_tail(seed, L, ray_o, ray_dir, info, batt, bpdf, attenuation, contribution, regularization, mx);
    }
    return contribution;
}

// tonemap_pixel (:753-771): ACES fit, sRGB curve, clamp, BGRA
PTG_D float aces(float c) { return (c * (2.51f * c + 0.03f)) / (c * (2.43f * c + 0.59f) + 0.14f); }
PTG_D float srgb(float c)
{
    return c < 0.0031308f ? c * 12.92f
                          : (float)(dpow((double)c, (double)(1.0f / 2.4f)) * (double)1.055f - (double)0.055f);
}
PTG_D uchar4 tonemap(f3 c)
{
    const float r = clampf(srgb(aces(c.x)), 0.0f, 1.0f);
    const float g = clampf(srgb(aces(c.y)), 0.0f, 1.0f);
    const float b = clampf(srgb(aces(c.z)), 0.0f, 1.0f);
    return make_uchar4((unsigned char)roundf(b * 255.0f), (unsigned char)roundf(g * 255.0f),
                       (unsigned char)roundf(r * 255.0f), 255);
}

} // namespace dm
} // namespace ptg
