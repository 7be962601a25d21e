// HIP kernels + C ABI of the GPU renderer (include/ptg.h).
//
//   k_pack_tris     indices + positions -> TriRec (48 B / triangle), + vertex attributes -> TriShade (128 B)
//   (BVH blocks are packed on the host, host/block_bvh.cpp)
//   k_trace         path_trace_pixel for a (pixel set x sample chunk) grid,
//                   one work-item per (pixel, sample); results to a
//                   [sample][pixel] float4 buffer in HBM
//   k_accumulate    baseline_render's j-ordered float32 sum over the chunk,
//                   then (last chunk) / SPP + tonemap_pixel (main.cc:24-43)
//   k_sample_list   path_trace_pixel for an explicit (x, y, j) list (parity)
//   k_rays          ray_query closest hit + shadow any-hit (parity)
//   k_tonemap, k_scatter_tiles
//
// No fallback path exists: every entry point fails loudly (negative code +
// ptg_last_error) when HIP or the device is unavailable.
#include <hip/hip_runtime.h>
#include "ptg.h"
#include "device/layout.h"
#include "device/path_tracer.h"
#include "device/wavefront.h"
#include "ptg_device.h"   // ptg_device_selftest, compiled here with the library's own flags (ptg_arith_selftest)
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <tuple>
#include <string>
#include <vector>
#include <unordered_map>
#include <unordered_set>
#include "host/block_bvh.h"
#include <vector>

namespace ptg {
void set_last_error(const std::string& msg);   // scene.cpp
}

using namespace ptg;
using namespace ptg::dm;

namespace {

constexpr int kBlock = 256;
#define PTG_SHADE_WAVES 3   // the certified pass (MathFast): 168 VGPRs, 6 spilled; the exact pass runs at 2
// the surface pass's math: MathFast (certified ocml + the exact redo pass) or
// MathExactLds (glibc's algorithms directly, no redo)
using ShadeMath = MathFast;

// ---------------------------------------------------------------- kernels --

// The aperture polygon's vertex directions of every subframe (regular_polygon,
// path_tracer.hh:50-62): (sin, cos) of side_radians * k + angle for
// k = 0 .. sides + 1.  A polygon has few vertices and every sample's camera
// ray uses two of them, so the camera kernel reads them instead of making
// four double-precision trig calls.  One thread per (subframe, k).
__global__ void k_polygon_table(const uint8_t* __restrict__ subframes, uint32_t count, float2* __restrict__ out)
{
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if(t >= count * kPolyStride) return;
    const uint32_t i = t / kPolyStride, k = t % kPolyStride;
    const uint8_t* cam = subframes + size_t(i) * SF_STRIDE + SF_CAM;
    const int32_t sides = (int32_t)rd_u(cam, 80);
    f2 v{0.0f, 0.0f};
    if(sides > 3 && (uint32_t)sides <= kPolyMaxSides && k <= (uint32_t)sides + 1u)
        v = polygon_vertex(rd_f(cam, 76), (uint32_t)sides, (float)k);
    out[t] = make_float2(v.x, v.y);
}

struct MeshJob {
    uint32_t index_offset, triangle_count, base_vertex_offset, pad;
};

// one thread per triangle of each new mesh: its TriRec (positions) and its
// TriShade (normals, albedos, materials), both at index_offset / 3 + t
__global__ void k_pack_tris(const uint32_t* __restrict__ indices, const float4* __restrict__ pos, TriRec* __restrict__ out,
                            const MeshJob* __restrict__ jobs, const float4* __restrict__ normal,
                            const float4* __restrict__ albedo, const float4* __restrict__ material,
                            TriShade* __restrict__ shade)
{
    const MeshJob j = jobs[blockIdx.y];
    for(uint32_t t = blockIdx.x * blockDim.x + threadIdx.x; t < j.triangle_count; t += gridDim.x * blockDim.x)
    {
        const uint32_t* tri = indices + j.index_offset + 3u * t;
        const float4 a = pos[j.base_vertex_offset + tri[0]];
        const float4 b = pos[j.base_vertex_offset + tri[1]];
        const float4 c = pos[j.base_vertex_offset + tri[2]];
        TriRec r;
        r.p0x = a.x; r.p0y = a.y; r.p0z = a.z; r.p1x = b.x;
        r.p1y = b.y; r.p1z = b.z; r.p2x = c.x; r.p2y = c.y;
        r.p2z = c.z; r.pad0 = 0; r.pad1 = 0; r.pad2 = 0;
        out[j.index_offset / 3u + t] = r;
        TriShade sh;
        for(int k = 0; k < 3; ++k)
        {
            const uint32_t v = j.base_vertex_offset + tri[k];
            const float4 n = normal[v], a = albedo[v], m = material[v];
            float* g = sh.v + 10 * k;
            g[0] = n.x; g[1] = n.y; g[2] = n.z;
            g[3] = a.x; g[4] = a.y; g[5] = a.z;
            g[6] = m.x; g[7] = m.y; g[8] = m.z; g[9] = m.w;
        }
        sh.v[30] = sh.v[31] = 0.0f;
        shade[j.index_offset / 3u + t] = sh;
    }
}

// Which image pixels a launch covers: a rectangle, or an interleaved tile set.
struct PixelMap {
    uint32_t tiles;                 // 0: rectangle, 1: tiles
    uint32_t x0, y0, w, h;          // rectangle
    uint32_t tw, th, tiles_x, first, stride;
    uint32_t img_w, img_h;
    uint32_t npix;

    __device__ __forceinline__ bool pixel(uint32_t p, uint32_t& x, uint32_t& y) const
    {
        if(!tiles)
        {
            x = x0 + p % w;
            y = y0 + p / w;
            return true;
        }
        const uint32_t per = tw * th;
        const uint32_t t = first + (p / per) * stride;
        const uint32_t q = p % per;
        x = (t % tiles_x) * tw + q % tw;
        y = (t / tiles_x) * th + q / tw;
        return x < img_w && y < img_h;
    }
};

// 16-byte non-temporal load / store of a float4 or uint4 record
template<typename T> __device__ __forceinline__ T nt_load(const T* p)
{
    typedef uint32_t v4u __attribute__((ext_vector_type(4)));
    const v4u v = __builtin_nontemporal_load(reinterpret_cast<const v4u*>(p));
    T out;
    __builtin_memcpy(&out, &v, 16);
    return out;
}
template<typename T> __device__ __forceinline__ void nt_store(T* p, T value)
{
    typedef uint32_t v4u __attribute__((ext_vector_type(4)));
    v4u v;
    __builtin_memcpy(&v, &value, 16);
    __builtin_nontemporal_store(v, reinterpret_cast<v4u*>(p));
}

__device__ __forceinline__ unsigned long long wave_sum(uint32_t v)
{
    unsigned long long s = v;
    for(int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
    return s;
}

// Counting builds only: wave-reduce the counters, one atomic per counter per wave.
__device__ __forceinline__ void flush_counters(const Counters& c, unsigned long long* dev, uint32_t samples)
{
    const unsigned long long v[8] = {wave_sum(samples), wave_sum(c.visits), wave_sum(c.tri_tests),
                                     wave_sum(c.blas_entries), wave_sum(c.queries), wave_sum(c.shades),
                                     wave_sum(c.tlas_visits), wave_sum(c.iters)};
    if((threadIdx.x & 63u) == 0)
        for(int k = 0; k < 8; ++k)
            if(v[k]) atomicAdd(dev + k, v[k]);
}

// Counting builds: paths the MathFast shading passes listed for the exact
// pass - [0] surface, [1] sky - then per certificate site (ref_math.h
// CertSite) the listed paths in which it failed (kRedoWords words).
constexpr int kRedoWords = 2 + CS_COUNT;
__device__ __forceinline__ void tally_redo(unsigned long long* tally, int kind, uint32_t fail_mask)
{
    atomicAdd(tally + kind, 1ull);
    for(int k = 0; k < CS_COUNT; ++k)
        if(fail_mask & (1u << k)) atomicAdd(tally + 2 + k, 1ull);
}

// ---- wavefront pipeline (csrc/device/wavefront.h) ----


// Lane -> (pixel, sample) of a chunk: a wave holds 8 pixels x 8 consecutive
// samples (one motion-blur subframe); consecutive waves walk the sample
// groups of one pixel group.
__device__ __forceinline__ void chunk_coords(uint32_t i, uint32_t nj, uint32_t& p, uint32_t& jj)
{
    const uint32_t wave = i >> 6, lane = i & 63u;
    const uint32_t sgroups = (nj + 7u) >> 3;
    jj = (wave % sgroups) * 8u + (lane & 7u);
    p = (wave / sgroups) * 8u + (lane >> 3);
}

// counts[2r]: paths queued for round r; counts[2r+1]: their pending NEE rays.
// Round 0 is every lane of the chunk in lane order (queue position = lane, no
// compaction); lanes outside the chunk or the image are queued as dead paths
// (an empty TLAS, retired by the first shade).
template<bool COUNT>
__global__ __launch_bounds__(kBlock) void k_wf_camera(DevScene sc, PixelMap pm, uint32_t j0, uint32_t nj, uint32_t M,
                                                      PathSoA S, uint32_t* __restrict__ counts, float4* __restrict__ out,
                                                      unsigned long long* __restrict__ counters)
{
    if(blockIdx.x == 0 && threadIdx.x == 0) counts[0] = M;
    uint32_t lives = 0;
    for(uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < M; i += gridDim.x * blockDim.x)
    {
        uint32_t p, jj, x = 0, y = 0;
        chunk_coords(i, nj, p, jj);
        const bool in_chunk = p < pm.npix && jj < nj;
        const bool live = in_chunk && pm.pixel(p, x, y);
        const uint32_t slot = in_chunk ? jj * pm.npix + p : 0xFFFFFFFFu;
        if(!live)
        {
            if(in_chunk) st_out(out + slot, make_float4(0.f, 0.f, 0.f, 0.f));
            st_state(S.meta + i, make_uint4(slot, META_DEAD, kBePop, 0u));   // no TLAS: the walk ends at once
            st_state(S.ray_o + i, make_float4(0.f, 0.f, 0.f, 0.f));
            st_state(S.ray_d + i, make_float4(0.f, 0.f, 1.f, 0.f));
            continue;
        }
        const int32_t j = (int32_t)(j0 + jj);
        const uint8_t* sf = subframe_of(sc, j);
        u4 seed;
        f3 o, d;
        camera_ray(sc, sf, x, y, j, seed, o, d);
        const uint32_t sub = (uint32_t)(sf - sc.subframes) / SF_STRIDE;
        st_state(S.meta + i, make_uint4(slot, meta_pack(0, false, sub), sc.tlas_root[sub], 0u));
        st_state(S.seed + i, to_uint4(seed));
        st_state(S.ray_o + i, make_float4(o.x, o.y, o.z, 0.f));
        st_state(S.ray_d + i, make_float4(d.x, d.y, d.z, 0.f));
        ++lives;
    }
    if(COUNT) flush_counters(Counters{}, counters, lives);
}

// BVH walks of one round over a queue: ANY = false walks the extension rays
// (closest hit, queue positions 0..n-1), ANY = true the pending NEE rays
// (any hit, positions from the NEE list).  Persistent "while-while" loop:
// the grid is sized to what is resident, each wave owns a contiguous range of
// the queue (no atomics), and a lane that finishes its ray takes the next one
// of its wave's range, so the wave never idles behind its longest ray.
#ifndef PTG_ANY_RUN
#define PTG_ANY_RUN 4
#endif
constexpr uint32_t kAnyRun = PTG_ANY_RUN;   // consecutive queue groups per run of the any-hit walk (k_wf_walk)
constexpr int kRefillIdle = 24;   // refill once at least this many lanes are idle (16 / 32: slower)
// waves per SIMD the walks are compiled for: the closest-hit walk at 96 VGPRs
// (104 uncapped, no spills at 96), the any-hit walk at 80 (76 used), so a
// shade wave (160) fits beside it
#define PTG_WALK_WAVES 5
#define PTG_SHADOW_WAVES 6
#define PTG_WALK_ATTR __attribute__((amdgpu_waves_per_eu(ANY ? PTG_SHADOW_WAVES : PTG_WALK_WAVES, 8)))
constexpr int kWalkUnroll = 2;     // node steps per leaf phase (1 and 3 measured slower)
// Walk residency per walk kind (closest hit, any hit): the LDS of a walk
// block is padded to 1 / kWalkResident of the CU's (0: not padded), and the
// grid holds kWalkBlocksPerCu blocks per CU (one resident wave, see
// ptg_context_create).  Timing knobs PTG_WALK_RESIDENT[_ANY] and
// PTG_WALK_BLOCKS[_ANY] override them (the results do not depend on them).
constexpr uint32_t kWalkResident[2] = {4, 0};
constexpr uint32_t kWalkBlocksPerCu[2] = {3, 3};
constexpr uint32_t kWfSlots = 2;           // concurrent wavefront chunk pipelines (ptg_context::Slot)
constexpr uint32_t kBands = 1024;   // XCD bands of a walk queue: a multiple of the XCD count (8 on MI355X)
// a chunk's device counters: per round the queue / NEE list lengths (2 words,
// plus 4 spare), the hit / sky list lengths (2), the redo list lengths (2)
constexpr uint32_t kCountWords(uint32_t rounds) { return 4 * (rounds + 2) + 2 * rounds; }
// a chunk pipeline's state bytes per queued path, as render_map carves them:
// 2 ping-pong PathSoA halves of 9 x 16 B, 2 TraceOut sets (hit 16 B, bary
// 8 B, shadow 4 B), 5 lists of 4 B (2 NEE lists, hit, sky, redo)
constexpr size_t kStateBytesPerPath = 2 * 9 * 16 + 2 * (16 + 8 + 4) + 5 * 4;
constexpr uint32_t kRedoGrid = 16;   // blocks of the MathExact shading passes (grid-stride over a short list)

// Walk statistics of the counting build (per walk kind, see WalkStats): how
// many lanes each vector-memory instruction of the walk serves.  The walk's
// vector-memory issue costs the same per wave instruction whatever its EXEC
// mask (profiles/r02_probe/ta_probe.txt), so lanes per instruction is the
// lever on that level.
enum WalkStat : int { WS_NODE_WAVES = 0, WS_NODE_LANES, WS_LEAF_WAVES, WS_LEAF_LANES, WS_REFILL_WAVES,
                      WS_REFILL_LANES, WS_ITERS, WS_ACTIVE_LANES, WS_COUNT };

template<bool ANY, bool COUNT>
__global__ __launch_bounds__(kBlock) PTG_WALK_ATTR void k_wf_walk(DevScene sc, PathSoA S, const uint32_t* __restrict__ counts,
                                                    uint32_t round, const uint32_t* __restrict__ list, TraceOut tr,
                                                    uint32_t nxcd, unsigned long long* __restrict__ counters,
                                                    unsigned long long* __restrict__ wstats)
{
    // the walks wait on memory most of their cycles: when a walk wave and a
    // shade / sky wave of the other pipeline are both ready on a SIMD, the
    // walk issues first (priorities 1-3 measured; 3: frame 0 -0.2%, frame
    // 450 -0.3%, profiles/r04m_prio/)
    __builtin_amdgcn_s_setprio(3);
    const uint32_t n = counts[2 * round + (ANY ? 1 : 0)];
    const uint32_t lane = threadIdx.x & 63u;
    // XCD-aware static split: the queue's 64-entry groups (8 pixels x 8
    // samples each) are cut into kBands bands dealt round-robin to the XCDs
    // (workgroup b runs on XCD b % nxcd), so each XCD's L2 serves a few image
    // bands instead of the whole frame.  Inside its bands, wave w of an XCD
    // takes the groups w, w + W, w + 2W, ...: every wave samples all of its
    // XCD's bands (balanced) and the waves in flight cover a narrow window.
    const uint32_t xcd = blockIdx.x % nxcd;
    const uint32_t waves = ((gridDim.x / nxcd) * blockDim.x) >> 6;
    const uint32_t wave = ((blockIdx.x / nxcd) * blockDim.x + threadIdx.x) >> 6;
    const uint32_t groups = (n + 63u) >> 6;
    const uint32_t band = max(1u, (groups + kBands - 1u) / kBands);
    const uint32_t local = (kBands / nxcd) * band;    // this XCD's group slots (some past the end)
    // The any-hit walk deals runs of kAnyRun consecutive groups per wave (wave
    // w: runs w, w + W, ...) instead of single groups: a wave's next group is
    // then usually the same pixels' next 8 samples (or the next pixels), so
    // the occluder its last group found (the candidate, try_candidate) lies on
    // the new rays' way to the sun too.  The closest-hit walk keeps runs of 1.
    // Runs only where they keep a run inside one band and still leave every
    // wave work (small queues - late rounds, small frames, tile renders - take
    // single groups: a run crossing bands would jump nxcd * band groups).
    static_assert((kAnyRun & (kAnyRun - 1u)) == 0, "kAnyRun is a power of two");
    const uint32_t rl = (ANY && band >= kAnyRun && groups >= waves * kAnyRun) ? uint32_t(__builtin_ctz(kAnyRun)) : 0u;
    const uint32_t R = 1u << rl;
    const uint32_t runs = (local + R - 1u) >> rl;
    const uint32_t end = wave < runs ? ((runs - wave + waves - 1) / waves) * R * 64u : 0u;
    uint32_t cursor = 0;
    const float tmin = (ANY || round > 0) ? MIN_RAY_DIST : 0.0f;
    const float tmax = ANY ? MAX_RAY_DIST : 1e9f;
    Counters cnt;
    // LDS: every lane's world ray, then the stack windows, one 64-lane x kCap
    // entry table per wave (ptg_context_create sizes the block's LDS)
    extern __shared__ WalkCold cold[];
    BlockWalker<LdsCold, typename WalkStackOf<ANY>::type> w;
    w.cold.c = (lds_cold_t*)(&cold[threadIdx.x]);   // C cast: generic -> LDS address space
    w.st.bind(cold + blockDim.x, threadIdx.x >> 6, lane, sc.spill + (size_t(blockIdx.x) * blockDim.x + threadIdx.x) * sc.spill_stride);
    bool active = false;
    uint32_t q = 0;
    // ANY: the wave's latest occluder (instance, triangle), wave-uniform (in
    // scalar registers): the candidate its next rays try first
    // (BlockWalker::try_candidate; a wave's rays come from one 8-pixel x
    // 8-sample group at a time, their shadow rays are nearly parallel)
    uint32_t occ_inst = 0xFFFFFFFFu, occ_prim = 0;
    // a finished walk writes its result: the shadow flag, or the closest hit;
    // results stream once through the caches (non-temporal), so they do not
    // evict BVH records from L2 / the Infinity Cache
    auto finish = [&](int r) {
        if(ANY) __builtin_nontemporal_store(r == 2 ? 1u : 0u, tr.shadow + q);
        else
        {
            const Hit h = w.result();
            // (primitive_id: the mesh-global triangle, LdsCold::kGlobalTri)
            nt_store(tr.hit + q, make_uint4(__float_as_uint(h.thit), h.instance_id, h.primitive_id, h.back_face ? 1u : 0u));
            if(h.instance_id != 0xFFFFFFFFu)   // a miss is shaded without its barycentrics
                __builtin_nontemporal_store(__builtin_bit_cast(unsigned long long, make_float2(h.bx, h.by)),
                                            reinterpret_cast<unsigned long long*>(tr.bary + q));
        }
    };
    unsigned long long ws[WS_COUNT] = {};   // COUNT: lane 0's tallies for its wave
    auto tally = [&](int waves_slot, bool loads) {
        const unsigned long long m = __ballot(loads);
        if(lane == 0 && m)
        {
            ws[waves_slot] += 1;
            ws[waves_slot + 1] += (unsigned long long)__popcll(m);
        }
    };
    for(;;)
    {
        if(cursor < end)
        {
            const unsigned long long idle = __ballot(!active);
            const uint32_t nidle = (uint32_t)__popcll(idle);
            if(nidle >= (uint32_t)kRefillIdle || nidle == 64u)
            {
                bool took = false;
                if(!active)
                {
                    const uint32_t v = cursor + (uint32_t)__popcll(idle & ((1ull << lane) - 1ull));
                    const uint32_t k = v >> 6;   // this wave's k-th group
                    const uint32_t l = (wave + (k >> rl) * waves) * R + (k & (R - 1u));
                    const uint32_t t = ((xcd + nxcd * (l / band)) * band + l % band) * 64u + (v & 63u);
                    if(v < end && l < local && t < n)
                    {
                        q = ANY ? list[t] : t;
#if PTG_DEBUG
                        // the NEE list names positions of this round's path queue
                        const bool bad = ANY && q >= counts[2 * round];
                        if(bad && sc.debug) atomicAdd(sc.debug + kDebugQueue, 1u);
                        if(!bad)
#endif
                        {
                            // path state streams once through the caches: non-temporal
                            const uint4 m = nt_load(S.meta + q);
                            w.init(m.z, xyz(nt_load(S.ray_o + q)),
                                   ANY ? xyz(nt_load(S.nee_d + q)) : xyz(nt_load(S.ray_d + q)), tmin, tmax);
                            if(ANY) w.try_candidate(sc, occ_inst, occ_prim, meta_sub(m));
                            active = true;
                            took = true;
                            if(COUNT) cnt.queries++;
                        }
                    }
                }
                if(COUNT) tally(WS_REFILL_WAVES, took);
                cursor = min(end, cursor + nidle);
            }
        }
        if(!__any(active)) break;
        if(COUNT)
        {
            const unsigned long long m = __ballot(active);
            if(lane == 0)
            {
                ws[WS_ITERS] += 1;
                ws[WS_ACTIVE_LANES] += (unsigned long long)__popcll(m);
                cnt.iters++;
            }
        }
        // Node phase, up to kWalkUnroll block steps (each after the pop it
        // needs), for lanes not standing at a leaf; then one leaf phase for the
        // lanes that are.  The leaf code (triangle test, BLAS entry) then runs
        // once per iteration with many lanes, not once per block step with few.
        int r = 0;
#pragma unroll
        for(int u = 0; u < kWalkUnroll; ++u)
        {
            if(COUNT) cnt.step_loads = 0;
            if(active && !w.at_leaf()) r = w.template node_step<COUNT>(sc, cnt);   // (a lane with a parked triangle walks on)
            if(COUNT) tally(WS_NODE_WAVES, (cnt.step_loads & 1u) != 0);
            if(active && r != 0)
            {   // ANY: after a candidate's instance, the TLAS (BlockWalker::resume_tlas)
                if(!(ANY && w.resume_tlas()))
                {
                    finish(r);
                    active = false;
                }
                r = 0;
            }
        }
        if(COUNT) cnt.step_loads = 0;
        bool occluded = false;
        if(active && w.wants_leaf())
        {
            r = w.template leaf_step<ANY, COUNT>(sc, cnt);
            occluded = ANY && r == 2;
            if(r != 0) { finish(r); active = false; }
        }
        if(ANY)
        {   // the wave's candidate becomes an occluder one of its lanes just found
            const unsigned long long om = __ballot(occluded);
            if(om)
            {
                const int l = __ffsll((long long)om) - 1;
                occ_inst = __builtin_amdgcn_readlane(w.inst, l);
                occ_prim = __builtin_amdgcn_readlane(w.cur, l);   // a walk that returned 2 left its occluder in cur
            }
        }
        if(COUNT) tally(WS_LEAF_WAVES, (cnt.step_loads & 6u) != 0);
    }
    if(COUNT)
    {
        flush_counters(cnt, counters, 0);
        if(lane == 0)
            for(int k = 0; k < WS_COUNT; ++k)
                if(ws[k]) atomicAdd(wstats + k, ws[k]);
    }
}

// Shading of one round is split by what the paths will run.
//
// k_wf_classify reads every queued path's trace result and deals the queue,
// 256 entries per block, into two lists through an LDS counting sort: paths
// whose ray hit a surface (shaded by k_wf_shade) and paths whose ray left the
// scene (shaded by k_wf_sky), each grouped by whether a pending NEE ray still
// has to be finished.  A wave then runs one of the long, mutually exclusive
// branches of shade_path, and the sky branch - the double-precision
// atmosphere integrals - runs in its own small kernel at high occupancy.
// Which lane shades which path has no effect on the result.
__global__ __launch_bounds__(kBlock) void k_wf_classify(const uint32_t* __restrict__ counts, uint32_t round, TraceOut tr,
                                                        uint32_t* __restrict__ hit_list,
                                                        uint32_t* __restrict__ sky_list, uint32_t* __restrict__ lcounts)
{
    // Each block deals a tile of kTile entries with ONE 64-bit atomic on the
    // packed (hit, sky) list lengths: a device-scope atomic is a fabric round
    // trip serialized per address, so their number, not the bytes, sets this
    // kernel's time.
    constexpr uint32_t kSub = 8, kTile = kSub * kBlock;
    const uint32_t n = counts[2 * round];
    __shared__ uint32_t bin_count[4];
    __shared__ unsigned long long base2;
    for(uint32_t tile = blockIdx.x * kTile; tile < n; tile += gridDim.x * kTile)
    {
        if(threadIdx.x < 4) bin_count[threadIdx.x] = 0;
        __syncthreads();
        uint32_t key[kSub], rank[kSub];
#pragma unroll
        for(uint32_t k = 0; k < kSub; ++k)
        {
            const uint32_t q = tile + k * kBlock + threadIdx.x;
            key[k] = 4u;
            rank[k] = 0;
            if(q < n)
            {
                const bool hit = __uint_as_float(tr.hit[q].x) > 0.0f;
                // shade(round-1) wrote 1 for survivors without a pending NEE ray,
                // the shadow walk 0/1 for those with one (meta is not read)
                const bool nee = round > 0 && tr.shadow[q] == 0;
                key[k] = (hit ? 2u : 0u) | (nee ? 1u : 0u);
                rank[k] = atomicAdd(&bin_count[key[k]], 1u);
            }
        }
        __syncthreads();
        if(threadIdx.x == 0)
        {
            const unsigned long long nsky = bin_count[0] + bin_count[1], nhit = bin_count[2] + bin_count[3];
            base2 = atomicAdd(reinterpret_cast<unsigned long long*>(lcounts), (nsky << 32) | nhit);
        }
        __syncthreads();
        const uint32_t hit_base = uint32_t(base2), sky_base = uint32_t(base2 >> 32);
#pragma unroll
        for(uint32_t k = 0; k < kSub; ++k)
        {
            const uint32_t q = tile + k * kBlock + threadIdx.x;
            if(key[k] == 4u) continue;
            if(key[k] & 2u) hit_list[hit_base + (key[k] == 3u ? bin_count[2] : 0u) + rank[k]] = q;
            else sky_list[sky_base + (key[k] == 1u ? bin_count[0] : 0u) + rank[k]] = q;
        }
        __syncthreads();   // bin_count is rewritten by the next tile
    }
}

// MISS: the caller shades a path whose ray left the scene (k_wf_classify put
// it on the sky list because its hit distance was not positive).  The walk
// reports such a ray as WalkerT::result() does, thit = -1 and no hit, and the
// sky branch of shade_path reads nothing else of it: the hit and barycentric
// records are not fetched (nor the barycentrics written by the walk).
template<bool MISS = false>
__device__ __forceinline__ void load_queued(const PathSoA& cur, const TraceOut& tr, uint32_t q, PathRec& p, Hit& h,
                                            bool& occluded, bool carried)
{
    p = load_path(cur, q, carried);
    occluded = meta_nee(p.meta) ? tr.shadow[q] != 0 : false;
    if(MISS)
    {
        h.thit = -1.0f;
        h.instance_id = 0xFFFFFFFFu;
        h.primitive_id = 0;
        h.back_face = false;
        h.bx = h.by = h.bz = 0.0f;
        return;
    }
    const uint4 hv = ld_state(tr.hit + q);
    // (bz = 1 - bx - by, the same float arithmetic as the walk's result())
    const float2 bv = __builtin_bit_cast(float2, __builtin_nontemporal_load(reinterpret_cast<const unsigned long long*>(tr.bary + q)));
    h.thit = __uint_as_float(hv.x);
    h.instance_id = hv.y;
    h.primitive_id = hv.z;
    h.back_face = hv.w != 0;
    h.bx = bv.x; h.by = bv.y; h.bz = 1.0f - bv.x - bv.y;
}

// A shading kernel's math policy (ref_math.h); MathExactLds copies glibc
// exp's table into the kernel's LDS array first (every thread, before any
// returns).
template<class MP>
__device__ __forceinline__ MP shading_policy(glibc::u2v* exp_tab)
{
    MP mp;
    if constexpr(MP::kLdsExp)
    {
        glibc::exp_table_to_lds((glibc::lds_u2v_t*)exp_tab);   // C cast: generic -> LDS address space
        __syncthreads();
        mp.xt = glibc::ExpTabLds{(const glibc::lds_u2v_t*)exp_tab};
    }
    (void)exp_tab;
    return mp;
}

// Surface hits: NEE finish, bounce tail, then NEE setup + BSDF sample of the
// next bounce or retire.  Survivors are appended per block (one atomic per
// queue per block), stored contiguously and grouped by the octant of their
// next ray, so the next round's 64-ray groups mostly walk one link order.
// MP = MathFast: ocml's double library with rounding certificates (ref_math.h);
// a path whose certificate failed is listed in redo_list (its length in
// redo_count) and shaded again by the MathExact instance, which takes
// redo_list as its hit_list (and appends nothing to a redo list).
template<bool COUNT, class MP>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(MP::kFast ? PTG_SHADE_WAVES : 2, 8))) void k_wf_shade(
    DevScene sc, PathSoA cur, PathSoA nxt, uint32_t* __restrict__ counts, uint32_t round, TraceOut tr,
    const uint32_t* __restrict__ hit_list, const uint32_t* __restrict__ lcounts, uint32_t* __restrict__ next_list,
    uint32_t* __restrict__ next_shadow, float4* __restrict__ out, uint32_t* __restrict__ redo_list,
    uint32_t* __restrict__ redo_count, unsigned long long* __restrict__ counters, unsigned long long* __restrict__ redo_tally)
{
    const uint32_t n = lcounts[0];
    Counters cnt;
    __shared__ uint32_t oct_count[8], oct_start[8], blk_base, nee_total, nee_base;
    __shared__ glibc::u2v exp_tab[MP::kLdsExp ? glibc::kExpTabEntries : 1];
    const MP mp0 = shading_policy<MP>(exp_tab);
    for(uint32_t base = blockIdx.x * blockDim.x; base < n; base += gridDim.x * blockDim.x)
    {
        const uint32_t i = base + threadIdx.x;
        bool cont = false, nee = false;
        PathRec p;
#if PTG_DEBUG
        const bool bad_q = i < n && hit_list[i] >= counts[2 * round];
        if(bad_q && sc.debug) atomicAdd(sc.debug + kDebugList, 1u);
        if(i < n && !bad_q)
#else
        if(i < n)
#endif
        {
            Hit h;
            bool occluded;
            const uint32_t q = hit_list[i];
            load_queued(cur, tr, q, p, h, occluded, round > 0);
            MP mp = mp0;
            const ShadeResult res = shade_path<COUNT, 1, MP>(sc, p, h, occluded, out, cnt, mp);
            if(MP::kFast && res == SH_REDO)
            {
                redo_list[atomicAdd(redo_count, 1u)] = q;
                if(COUNT) tally_redo(redo_tally, 0, mp.fail_mask);
            }
            cont = res == SH_CONTINUE;
            nee = cont && meta_nee(p.meta);
        }
        if(threadIdx.x < 8) oct_count[threadIdx.x] = 0;
        if(threadIdx.x == 8) nee_total = 0;
        __syncthreads();
        const uint32_t okey = cont ? octant(p.ray_d) : 0u;
        const uint32_t orank = cont ? atomicAdd(&oct_count[okey], 1u) : 0u;
        const uint32_t nrank = nee ? atomicAdd(&nee_total, 1u) : 0u;
        __syncthreads();
        if(threadIdx.x == 0)
        {   // one 64-bit atomic on the packed (queue, NEE list) lengths
            unsigned long long total = 0;
            for(int k = 0; k < 8; ++k) { oct_start[k] = uint32_t(total); total += oct_count[k]; }
            const unsigned long long old =
                (total | nee_total)
                    ? atomicAdd(reinterpret_cast<unsigned long long*>(&counts[2 * (round + 1)]),
                                (uint64_t(nee_total) << 32) | total)
                    : 0ull;
            blk_base = uint32_t(old);
            nee_base = uint32_t(old >> 32);
        }
        __syncthreads();
        const uint32_t qn = blk_base + oct_start[okey] + orank;
        if(cont) store_path(nxt, qn, p);
        if(nee) next_list[nee_base + nrank] = qn;
        else if(cont) __builtin_nontemporal_store(1u, next_shadow + qn);   // no NEE ray: k_wf_classify reads "occluded"
        __syncthreads();   // the LDS tables are rewritten by the next iteration
    }
    if(COUNT) flush_counters(cnt, counters, 0);
}

// Rays that left the scene: sun disk, NEE finish, the atmosphere integrals
// (path_tracer.hh:456-588), retire.  No survivors.  The atmosphere is exp
// work end to end, and here glibc's restated exp (its table copied to LDS)
// beats ocml's plus rounding certificates (MathFast: 2x the code, spills at
// 5 waves; measured DESIGN.md section 4), so this pass is exact by itself.
#define PTG_SKY_WAVES 5     // 96 VGPRs (10 spilled); 4 waves: 103, none - 5 measured 0.26% faster on frames 0 and 450 (profiles/r04q_tune/ab_sky5.log)
template<bool COUNT>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(PTG_SKY_WAVES, 8))) void k_wf_sky(
    DevScene sc, PathSoA cur, TraceOut tr, uint32_t round, const uint32_t* __restrict__ sky_list,
    const uint32_t* __restrict__ lcounts, float4* __restrict__ out, unsigned long long* __restrict__ counters)
{
    const uint32_t n = lcounts[1];
    Counters cnt;
    __shared__ glibc::u2v exp_tab[glibc::kExpTabEntries];
    MathExactLds mp = shading_policy<MathExactLds>(exp_tab);
    for(uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x)
    {
#if PTG_DEBUG
        if(sky_list[i] >= lcounts[0] + lcounts[1])   // positions of this round's queue (hits + sky)
        {
            if(sc.debug) atomicAdd(sc.debug + kDebugList, 1u);
            continue;
        }
#endif
        PathRec p;
        Hit h;
        bool occluded;
        load_queued<true>(cur, tr, sky_list[i], p, h, occluded, round > 0);
        shade_path<COUNT, 2>(sc, p, h, occluded, out, cnt, mp);
    }
    if(COUNT) flush_counters(cnt, counters, 0);
}

// One work-item per (pixel, sample).  A wave holds 8 pixels x 8 consecutive
// samples (one motion-blur subframe): lanes 0-7 are samples j..j+7 of pixel 0,
// and so on.  Consecutive waves walk the sample groups of one pixel group, so
// the waves in flight on a CU trace nearby pixels through the same TLASes.
template<bool COUNT>
__global__ __launch_bounds__(kBlock) void k_trace(DevScene sc, PixelMap pm, uint32_t j0, uint32_t nj,
                                                  float4* __restrict__ out, unsigned long long* __restrict__ counters)
{
    const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t wave = g >> 6, lane = g & 63u;
    const uint32_t sgroups = (nj + 7u) >> 3;
    const uint32_t sg = wave % sgroups, pg = wave / sgroups;
    const uint32_t jj = sg * 8u + (lane & 7u);
    const uint32_t p = pg * 8u + (lane >> 3);
    Counters cnt;
    if(p < pm.npix && jj < nj)
    {
        uint32_t x, y;
        float4 r = make_float4(0.f, 0.f, 0.f, 0.f);
        if(pm.pixel(p, x, y))
        {
            const f3 c = path_trace_sample<COUNT>(sc, x, y, (int32_t)(j0 + jj), cnt);
            r = make_float4(c.x, c.y, c.z, 0.f);
        }
        out[size_t(jj) * pm.npix + p] = r;
    }
    if(COUNT) flush_counters(cnt, counters, (p < pm.npix && jj < nj) ? 1u : 0u);
}

// acc[p] (+)= samples in index order; on the last chunk / spp and tonemap.
__global__ __launch_bounds__(kBlock) void k_accumulate(PixelMap pm, uint32_t nj, const float4* __restrict__ samples,
                                                       float4* __restrict__ acc, int first, int last, float spp,
                                                       float4* __restrict__ out_accum, uchar4* __restrict__ out_bgra)
{
    const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
    if(p >= pm.npix) return;
    float ax = 0.0f, ay = 0.0f, az = 0.0f;
    if(!first)
    {
        const float4 a = acc[p];
        ax = a.x; ay = a.y; az = a.z;
    }
    for(uint32_t j = 0; j < nj; ++j)
    {
        const float4 s = ld_out(samples + size_t(j) * pm.npix + p);
        ax = ax + s.x;
        ay = ay + s.y;
        az = az + s.z;
    }
    if(!last)
    {
        acc[p] = make_float4(ax, ay, az, 0.f);
        return;
    }
    ax = ax / spp;
    ay = ay / spp;
    az = az / spp;
    uint32_t x, y;
    const bool inside = pm.pixel(p, x, y);
    if(out_accum) out_accum[p] = inside ? make_float4(ax, ay, az, 0.f) : make_float4(0.f, 0.f, 0.f, 0.f);
    if(out_bgra) out_bgra[p] = inside ? tonemap(V3(ax, ay, az)) : make_uchar4(0, 0, 0, 0);
}

__global__ __launch_bounds__(kBlock) void k_sample_list(DevScene sc, uint32_t n, const uint2* __restrict__ xy,
                                                        const int32_t* __restrict__ js, float4* __restrict__ out)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if(i >= n) return;
    Counters cnt;
    const f3 c = path_trace_sample<false>(sc, xy[i].x, xy[i].y, js[i], cnt);
    out[i] = make_float4(c.x, c.y, c.z, 0.f);
}

__global__ __launch_bounds__(kBlock) void k_rays(DevScene sc, uint32_t tlas_root, uint32_t n,
                                                 const float* __restrict__ rays, uint32_t* __restrict__ hits)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if(i >= n) return;
    const float* r = rays + size_t(i) * 8;
    const f3 o = V3(r[0], r[1], r[2]), d = V3(r[3], r[4], r[5]);
    Counters cnt;
    Hit h, unused;
    trace<false, false>(sc, tlas_root, 0, o, d, r[6], r[7], h, cnt);
    const bool shadow = trace<true, false>(sc, tlas_root, 0, o, d, r[6], r[7], unused, cnt);
    uint32_t* w = hits + size_t(i) * 8;
    w[0] = __float_as_uint(h.bx);
    w[1] = __float_as_uint(h.by);
    w[2] = __float_as_uint(h.bz);
    w[3] = __float_as_uint(h.thit);
    w[4] = h.instance_id;
    w[5] = h.primitive_id;
    w[6] = h.back_face ? 1u : 0u;
    w[7] = shadow ? 1u : 0u;
}

__global__ void k_tonemap(uint32_t n, const float4* __restrict__ in, uchar4* __restrict__ out)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if(i < n) out[i] = tonemap(V3(in[i].x, in[i].y, in[i].z));
}

__global__ void k_scatter_tiles(PixelMap pm, const uchar4* __restrict__ tiles, uchar4* __restrict__ image)
{
    const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
    if(p >= pm.npix) return;
    uint32_t x, y;
    if(pm.pixel(p, x, y)) image[size_t(y) * pm.img_w + x] = tiles[p];
}

// ---------------------------------------------------------------- runtime --

struct DevBuf {
    void* p = nullptr;
    size_t bytes = 0;
    ~DevBuf() { if(p) (void)hipFree(p); }
    hipError_t reserve(size_t n)
    {
        if(n <= bytes && p) return hipSuccess;
        if(p) { (void)hipFree(p); p = nullptr; bytes = 0; }
        if(n == 0) return hipSuccess;
        hipError_t e = hipMalloc(&p, n);
        if(e == hipSuccess) bytes = n;
        return e;
    }
    template<typename T> T* as() const { return static_cast<T*>(p); }
};

// Pinned host staging for asynchronous uploads; `done` marks the end of the
// copies that last read it.
struct HostStage {
    void* p = nullptr;
    size_t bytes = 0;
    hipEvent_t done = nullptr;
    ~HostStage()
    {
        if(done)
        {
            (void)hipEventSynchronize(done);
            (void)hipEventDestroy(done);
        }
        if(p) (void)hipHostFree(p);
    }
    // waits for the copies that last read it, then grows it to n bytes
    hipError_t reserve(size_t n)
    {
        if(!done)
            if(hipError_t e = hipEventCreateWithFlags(&done, hipEventDisableTiming)) return e;
        if(hipError_t e = hipEventSynchronize(done)) return e;
        if(n <= bytes && p) return hipSuccess;
        if(p) { (void)hipHostFree(p); p = nullptr; bytes = 0; }
        hipError_t e = hipHostMalloc(&p, std::max<size_t>(n, 1), hipHostMallocDefault);
        if(e == hipSuccess) bytes = std::max<size_t>(n, 1);
        return e;
    }
};

int hip_fail(hipError_t e, const char* what)
{
    set_last_error(std::string(what) + ": " + hipGetErrorName(e) + " (" + hipGetErrorString(e) + ")");
    return PTG_E_HIP;
}

#define PTG_HIP(call)                                                        \
    do {                                                                     \
        hipError_t e_ = (call);                                              \
        if(e_ != hipSuccess) return hip_fail(e_, #call);                     \
    } while(0)

int fail(int code, const std::string& msg)
{
    set_last_error(msg);
    return code;
}

uint32_t grid_for(size_t n, uint32_t block = kBlock) { return uint32_t((n + block - 1) / block); }

} // namespace

struct ptg_context {
    int device = 0;
    hipStream_t stream = nullptr;
    bool counting = false;
    // static scene: the shading arrays in reference layout, the triangle
    // records, and a host copy of the BLAS nodes + links (packed into blocks
    // when an instance first names a BLAS)
    DevBuf indices, pos, normal, albedo, material, tris, tri_shade;
    std::vector<ptg_bvh_node> host_nodes;
    std::vector<ptg_bvh_link> host_links;
    std::vector<uint32_t> host_indices;    // the mesh arrays the occluder candidates' leaf boxes are checked against
    std::vector<ptg_float3> host_pos;
    // per (BLAS, mesh): every BLAS leaf's box is its triangle's vertex bounds
    // (bvh.cc:243-246), so a candidate triangle's leaf box can be computed from
    // its vertices (k_wf_walk<ANY>); checked once per pair on the host
    std::map<std::tuple<uint32_t, uint32_t, uint32_t>, bool> leaf_bounds_ok;
    size_t static_nodes = 0, index_count = 0, vertex_count = 0;
    std::unordered_set<uint32_t> packed_mesh;
    // BLAS blocks packed so far (host copy; their device copy leads `blocks`)
    BlockCache cache;
    size_t blas_on_device = 0;                           // leading cache.blas entries already in `blocks`
    bool scene_ready = false;
    // frame: blocks = [BLAS blocks][this frame's TLAS blocks]
    DevBuf blocks, tlas_root, subframes, inst_trav, inst_shade, inst_box, jobs, polygon, spill;
    HostStage stage[2];                                  // ptg_upload_frame's pinned staging, used alternately
    uint32_t stage_next = 0;
    size_t block_count = 0, subframe_count = 0, instance_count = 0;
    uint32_t stack_bound = 0;                            // TLAS + BLAS stack bound of this frame (entries)
    bool attrs_finite = false;                           // every vertex albedo / material value finite
    std::vector<uint32_t> host_tlas_root;
    std::vector<ptg_subframe> host_subframes;
    bool frame_ready = false;
    // render workspace
    DevBuf samples, acc, tmp_a, tmp_b, tmp_c, counters;
    DevBuf debug;                          // PTG_DEBUG builds: kDebugSlots violation counters
    uint64_t last_counters[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    // k_trace launch timing (HIP events on the launch stream)
    bool timing = false;
    std::vector<hipEvent_t> ev_start, ev_stop;
    std::vector<int> ev_kind;
    size_t ev_used = 0;
    // 0: wavefront pipeline (default), 1: megakernel
    int pipeline = 0;
    uint32_t persistent_blocks = 2048;
    uint32_t walk_grid[2] = {2048, 2048};
    uint32_t walk_xcds[2] = {1, 1};        // XCDs the walk grid is dealt over (8 when the grid divides evenly)
    uint32_t walk_lds[2] = {0, 0};         // dynamic LDS per walk block: cold state + stack rings, padded to cap residency
    uint32_t hbm_pct = 35;                 // wavefront state: at most this share of HBM per chunk pipeline (ptg_set_hbm_share)
    // wavefront: <= 2^chunk_log2 live paths per chunk.  2^27 paths x 380 B
    // (kStateBytesPerPath 364 + the 16 B sample) = 51 GB per pipeline, ~35% of an MI355X's HBM for the two pipelines
    // together, so a default render leaves most of the GPU to other tenants;
    // 2^28 (~71%) is 1-3% faster on a GPU the renderer owns alone.
    uint32_t chunk_log2 = 27;
    DevBuf wf_state;
    uint64_t kind_counters[6][8] = {};
    uint64_t walk_stats[2][8] = {};        // counting builds: WalkStat tallies of the closest-hit / any-hit walks
    uint64_t redo_stats[kRedoWords] = {};  // counting builds: the certified shading's redo tallies (tally_redo)
    // second stream for the sky kernels + the events that order it with `stream`
    hipStream_t side = nullptr;
    hipEvent_t ev_main = nullptr, ev_side = nullptr;
    // Wavefront chunk pipelines ("slots").  With two slots, consecutive
    // chunks run concurrently on their own stream pairs and buffers, so one
    // chunk's round-0 walk and shade overlap the other's sky and shadow
    // kernels; k_accumulate still folds the chunks in sample order, each on
    // its chunk's slot stream, chained by events across the slots (render_map).
    // Slot 0 is the context's own stream pair and buffers.
    struct Slot {
        hipStream_t main = nullptr, side = nullptr;
        hipEvent_t ev_main = nullptr, ev_side = nullptr, ev_acc = nullptr;   // ev_acc: its last fold done
        DevBuf own_state, own_samples;
        DevBuf* state = nullptr;
        DevBuf* samples = nullptr;
    };
    static constexpr uint32_t kMaxSlots = kWfSlots;
    Slot slot[kMaxSlots];
    uint32_t nslots = 1;
    uint32_t concurrency = 2;              // ptg_set_concurrency
    hipEvent_t ev_render_start = nullptr;
    ~ptg_context()
    {
        if(ev_main) (void)hipEventDestroy(ev_main);
        if(ev_side) (void)hipEventDestroy(ev_side);
        if(side) (void)hipStreamDestroy(side);
        for(uint32_t k = 1; k < kMaxSlots; ++k)
        {
            Slot& b = slot[k];
            for(hipEvent_t e: {b.ev_main, b.ev_side})
                if(e) (void)hipEventDestroy(e);
            for(hipStream_t st: {b.main, b.side})
                if(st) (void)hipStreamDestroy(st);
        }
        for(uint32_t k = 0; k < kMaxSlots; ++k)
        {
            if(slot[k].ev_acc) (void)hipEventDestroy(slot[k].ev_acc);
        }
        if(ev_render_start) (void)hipEventDestroy(ev_render_start);
        for(hipEvent_t e: ev_start) (void)hipEventDestroy(e);
        for(hipEvent_t e: ev_stop) (void)hipEventDestroy(e);
    }

    // Wait for everything queued on the context's streams: the caller's
    // stream, the second streams and the extra chunk pipeline.
    hipError_t drain() const
    {
        for(hipStream_t st: {stream, side})
            if(hipError_t e = hipStreamSynchronize(st)) return e;
        for(uint32_t k = 1; k < kMaxSlots; ++k)
            for(hipStream_t st: {slot[k].main, slot[k].side})
                if(st)
                    if(hipError_t e = hipStreamSynchronize(st)) return e;
        return hipSuccess;
    }
    // Grow a workspace buffer.  Growing frees the old allocation, which work
    // still queued on the context's streams may read: drain them first (rare,
    // the buffers only grow), rather than rely on hipFree's implicit sync.
    hipError_t grow(DevBuf& b, size_t n) const
    {
        if(n <= b.bytes && b.p) return hipSuccess;
        if(b.p)
            if(hipError_t e = drain()) return e;
        return b.reserve(n);
    }

    DevScene scene_args(const ptg_render_config* cfg) const
    {
        DevScene s;
        s.blocks = blocks.as<BlockCopy>();
        s.tlas_root = tlas_root.as<uint32_t>();
        s.tris = tris.as<TriRec>();
        s.tri_shade = tri_shade.as<TriShade>();
        s.inst_trav = inst_trav.as<InstTrav>();
        s.inst_shade = inst_shade.as<InstShade>();
        s.inst_box = inst_box.as<InstBox>();
        s.indices = indices.as<uint32_t>();
        s.normal = normal.as<float>();
        s.albedo = albedo.as<float>();
        s.material = material.as<float>();
        s.subframes = subframes.as<uint8_t>();
        s.polygon = polygon.as<float2>();
        s.width = cfg ? cfg->width : 0;
        s.height = cfg ? cfg->height : 0;
        s.spp = cfg ? cfg->samples_per_pixel : 0;
        s.max_bounces = cfg ? cfg->max_bounces : 0;
        s.student_id = cfg ? cfg->student_id : 0;
        s.blur_step = cfg ? cfg->samples_per_motion_blur_step : 8;
        s.subframe_count = uint32_t(subframe_count);
        s.block_count = uint32_t(block_count);
        s.spill = nullptr;
        s.spill_stride = stack_bound;
        s.tri_count = uint32_t(index_count / 3);
        s.inst_count = uint32_t(instance_count);
        s.debug = PTG_DEBUG ? debug.as<uint32_t>() : nullptr;
        s.attrs_finite = attrs_finite ? 1u : 0u;
        return s;
    }
};

namespace {

int bind(ptg_context* ctx)
{
    if(!ctx) return fail(PTG_E_INVALID, "null context");
    PTG_HIP(hipSetDevice(ctx->device));
    return PTG_OK;
}

int check_cfg(const ptg_context* ctx, const ptg_render_config* cfg, uint32_t sample_end)
{
    if(!cfg || cfg->width == 0 || cfg->height == 0 || cfg->samples_per_pixel == 0 || cfg->samples_per_motion_blur_step == 0)
        return fail(PTG_E_INVALID, "bad render config");
    if(!ctx->scene_ready || !ctx->frame_ready) return fail(PTG_E_INVALID, "scene/frame not uploaded");
    if(sample_end > 0)
    {
        const uint64_t need = (uint64_t(sample_end) - 1) / cfg->samples_per_motion_blur_step + 1;
        if(need > ctx->subframe_count)
            return fail(PTG_E_RANGE, "sample range needs " + std::to_string(need) + " subframes, frame has " +
                                         std::to_string(ctx->subframe_count));
    }
    if(uint64_t(cfg->width) * cfg->height > (1ull << 31)) return fail(PTG_E_RANGE, "image too large");
    return PTG_OK;
}

// Kernel kinds for timing and work counters.
// (work counters use the first K_KINDS; the sky and classify kernels are timed
// separately and count into K_SHADE)
enum Kind : int { K_MEGA = 0, K_EXTEND = 1, K_SHADOW = 2, K_SHADE = 3, K_CAMERA = 4, K_ACCUM = 5, K_KINDS = 6,
                  K_SKY = 6, K_CLASSIFY = 7 };
// counting builds: 8 work counters per kind, then WS_COUNT walk statistics
// for the closest-hit and the any-hit walk
// counting builds' device counters: 8 per kernel kind, the walk statistics,
// then the certified shading's redo tallies (kRedoWords, tally_redo)
constexpr int kCounterWords = K_KINDS * 8 + 2 * WS_COUNT + kRedoWords;

int timed_begin(ptg_context* ctx, int kind, hipStream_t st = nullptr);
int timed_end(ptg_context* ctx, hipStream_t st = nullptr);

// Render the pixels of `pm` for samples [j0, j1): per chunk of samples, the
// path kernels write one float4 per (pixel, sample); k_accumulate folds the
// chunk into the running per-pixel sum in sample order.
int render_map(ptg_context* ctx, const ptg_render_config* cfg, PixelMap pm, uint32_t j0, uint32_t j1,
               ptg_float4* out_accum, ptg_uchar4* out_bgra)
{
    if(pm.npix == 0) return PTG_OK;
    if(j1 <= j0) return fail(PTG_E_INVALID, "empty sample range");
    const bool wf = ctx->pipeline == 0;
    if(!wf && ctx->stack_bound >= PrivStack::kCap)
        return fail(PTG_E_RANGE, "the megakernel's walk stack holds " + std::to_string(PrivStack::kCap) +
                                     " entries, this frame's BVHs need " + std::to_string(ctx->stack_bound));
    // samples per chunk: megakernel <= 1 GiB of results; wavefront ~16 M live paths
    // Wavefront chunks are as large as HBM allows (capped at 35% of it): every
    // bounce round then launches over a long queue, so the walk and shade
    // launches run at full occupancy with short tails.  2^28 paths = 93 GB.
    // wavefront chunk pipelines: slot 0 is the context's stream pair and buffers
    const uint32_t nslots = (wf && ctx->concurrency >= 2) ? ctx->nslots : 1u;
    ptg_context::Slot* slots = ctx->slot;
    slots[0].main = ctx->stream;
    slots[0].side = ctx->side;
    slots[0].ev_main = ctx->ev_main;
    slots[0].ev_side = ctx->ev_side;
    slots[0].state = &ctx->wf_state;
    slots[0].samples = &ctx->samples;
    for(uint32_t k = 1; k < ptg_context::kMaxSlots; ++k)
    {
        slots[k].state = &slots[k].own_state;
        slots[k].samples = &slots[k].own_samples;
    }
    size_t target = (size_t(1) << 30) / sizeof(float4);
    if(wf)
    {
        size_t free_b = 0, total_b = 0;
        PTG_HIP(hipMemGetInfo(&free_b, &total_b));
        const size_t per_path = kStateBytesPerPath + sizeof(float4);   // + the path's per-sample result
        // a slot's share of HBM, but never more than what is actually free (other
        // tenants, torch's cache): buffers this context already holds count as free
        size_t held = 0;
        for(uint32_t k = 0; k < nslots; ++k)
            held += slots[k].state->bytes + slots[k].samples->bytes;
        const size_t share = total_b / 100 * (nslots > 2 ? ctx->hbm_pct * 2 / nslots : ctx->hbm_pct);
        const size_t avail = (free_b + held) / 100 * 85 / nslots;
        target = std::max<size_t>(size_t(1) << 16, std::min(size_t(1) << ctx->chunk_log2, std::min(share, avail) / per_path));
    }
    // equal chunks of whole motion-blur groups (multiples of 8 samples), each <= target paths
    const uint32_t span = j1 - j0;
    const uint32_t max_chunk = std::max<uint32_t>(8, uint32_t(std::min<size_t>(target / size_t(pm.npix), span)) & ~7u);
    uint32_t nchunks = (span + max_chunk - 1) / max_chunk;
    if(nslots > 1 && span >= 16u)
        nchunks = (std::max(nchunks, nslots) + nslots - 1) / nslots * nslots;   // whole rounds over the slots
    uint32_t chunk = std::min<uint32_t>(span, ((span + nchunks - 1) / nchunks + 7) & ~7u);
    const size_t M = size_t((pm.npix + 7) / 8) * ((chunk + 7) / 8) * 64;   // lanes per chunk (upper bound)
    if(M >= (1ull << 31)) return fail(PTG_E_RANGE, "chunk too large");
    for(uint32_t k = 0; k < nslots; ++k)
        PTG_HIP(ctx->grow(*slots[k].samples, size_t(pm.npix) * chunk * sizeof(float4)));
    PTG_HIP(ctx->grow(ctx->acc, size_t(pm.npix) * sizeof(float4)));
    unsigned long long* cnt_dev = nullptr;
    if(ctx->counting)
    {
        PTG_HIP(ctx->grow(ctx->counters, kCounterWords * sizeof(unsigned long long)));
        PTG_HIP(hipMemsetAsync(ctx->counters.p, 0, kCounterWords * sizeof(unsigned long long), ctx->stream));
        cnt_dev = ctx->counters.as<unsigned long long>();
    }
    const uint32_t rounds = cfg->max_bounces + 1;
    // path state of a slot: 2 x 9 records of 16 B per path, + trace outputs + NEE lists
    struct SlotState {
        PathSoA S[2];
        TraceOut trs[2] = {};   // per round parity: the sky kernel of round r reads its set while round r+1 writes the other
        uint32_t* lists[2] = {nullptr, nullptr};
        uint32_t *hit_list = nullptr, *sky_list = nullptr;   // this round's paths by shading kernel
        uint32_t* redo_hit = nullptr;   // surface paths to shade again with MathExact
        uint32_t* counts = nullptr;
    } st[ptg_context::kMaxSlots];
    if(wf)
        for(uint32_t k = 0; k < nslots; ++k)
        {
            const size_t rec = M * 16;
            PTG_HIP(ctx->grow(*slots[k].state, M * kStateBytesPerPath + kCountWords(rounds) * 4 + 256));
            char* b = slots[k].state->as<char>();
            SlotState& t = st[k];
            for(int h = 0; h < 2; ++h)
            {
                t.S[h].meta = reinterpret_cast<uint4*>(b); b += rec;
                t.S[h].seed = reinterpret_cast<uint4*>(b); b += rec;
                t.S[h].ray_o = reinterpret_cast<float4*>(b); b += rec;
                t.S[h].ray_d = reinterpret_cast<float4*>(b); b += rec;
                t.S[h].att = reinterpret_cast<float4*>(b); b += rec;
                t.S[h].contrib = reinterpret_cast<float4*>(b); b += rec;
                t.S[h].batt = reinterpret_cast<float4*>(b); b += rec;
                t.S[h].nee_c = reinterpret_cast<float4*>(b); b += rec;
                t.S[h].nee_d = reinterpret_cast<float4*>(b); b += rec;
            }
            for(TraceOut& o: t.trs)
            {
                o.hit = reinterpret_cast<uint4*>(b); b += M * 16;
                o.bary = reinterpret_cast<float2*>(b); b += M * 8;
                o.shadow = reinterpret_cast<uint32_t*>(b); b += M * 4;
            }
            t.lists[0] = reinterpret_cast<uint32_t*>(b); b += M * 4;
            t.lists[1] = reinterpret_cast<uint32_t*>(b); b += M * 4;
            t.hit_list = reinterpret_cast<uint32_t*>(b); b += M * 4;
            t.sky_list = reinterpret_cast<uint32_t*>(b); b += M * 4;
            t.redo_hit = reinterpret_cast<uint32_t*>(b); b += M * 4;
            t.counts = reinterpret_cast<uint32_t*>(b);
        }
    if(nslots > 1)
    {   // the other slot and the accumulation stream start after what the caller queued
        PTG_HIP(hipEventRecord(ctx->ev_render_start, ctx->stream));
        for(uint32_t k = 1; k < nslots; ++k)
            PTG_HIP(hipStreamWaitEvent(slots[k].main, ctx->ev_render_start, 0));
    }
    const DevScene sc = ctx->scene_args(cfg);
    // walk stack spill areas: one per (chunk pipeline, walk kind), since up to
    // four walk launches run at once; stack_bound entries per walk lane
    const size_t spill_region = size_t(std::max(ctx->walk_grid[0], ctx->walk_grid[1])) * kBlock * ctx->stack_bound;
    if(wf) PTG_HIP(ctx->grow(ctx->spill, std::max<size_t>(1, 2 * nslots * spill_region) * sizeof(uint2)));
    auto walk_scene = [&](uint32_t slot, int kind) {
        DevScene w = sc;
        w.spill = ctx->spill.as<uint2>() + (2 * slot + uint32_t(kind)) * spill_region;
        return w;
    };
    const uint32_t persistent = ctx->persistent_blocks;
    const bool overlap = wf && ctx->side != nullptr && ctx->concurrency >= 1;
    auto cnt_for = [&](int kind) { return cnt_dev ? cnt_dev + 8 * kind : nullptr; };
    auto ws_for = [&](bool any) { return cnt_dev ? cnt_dev + 8 * K_KINDS + (any ? WS_COUNT : 0) : nullptr; };
    unsigned long long* const redo_tally = cnt_dev ? cnt_dev + 8 * K_KINDS + 2 * WS_COUNT : nullptr;
    // The chunk plan: (first sample, samples, slot), in sample order (the
    // order the chunks are folded): equal chunks dealt round-robin.
    // PTG_STAGGER builds, with two slots: staggered - slot 1 starts and ends with half a chunk,
    // so the two pipelines never change chunks at the same moment (a change
    // runs the previous chunk's fold and the next chunk's camera kernel, with
    // no walk of that slot in flight: when both slots changed together the
    // GPU ran no walk for ~8 ms, profiles/r06c_timeline/).  The sample ranges
    // follow the chunks' expected completion order (equal cost per sample),
    // so each slot's next chunk finds its previous chunk already folded.
    struct Piece { uint32_t j, n, slot; };
    std::vector<Piece> plan;
#ifndef PTG_STAGGER
#define PTG_STAGGER 0   // 1: the staggered plan (measured 1-3% slower: its half chunks' rounds cost more than the gap they remove)
#endif
    if(PTG_STAGGER && nslots == 2 && chunk >= 16 && chunk % 16 == 0 && span > chunk)
    {
        struct Nominal { uint64_t done; uint32_t slot, n; };
        std::vector<Nominal> nom;
        // each slot takes half of the span; slot 1's first piece is half a chunk
        const uint32_t span1 = (span / 2) & ~7u, span0 = span - span1;
        uint64_t t = 0;
        for(uint32_t left = span0; left > 0;)
        {
            const uint32_t n = std::min(chunk, left);
            t += n;
            nom.push_back({t, 0u, n});
            left -= n;
        }
        t = 0;
        for(uint32_t left = span1, first = 1; left > 0; first = 0)
        {
            const uint32_t n = std::min(first ? chunk / 2 : chunk, left);
            t += n;
            nom.push_back({t, 1u, n});
            left -= n;
        }
        std::stable_sort(nom.begin(), nom.end(), [](const Nominal& a, const Nominal& b) {
            return a.done < b.done || (a.done == b.done && a.slot < b.slot); });
        uint32_t j = j0;
        for(const Nominal& x: nom)
        {
            if(j >= j1) break;
            const uint32_t n = std::min(x.n, j1 - j);
            plan.push_back({j, n, x.slot});
            j += n;
        }
        if(j != j1) plan.clear();   // (never: the pieces cover span0 + span1 = span)
    }
    if(plan.empty())
        for(uint32_t j = j0, k = 0; j < j1; j += chunk, ++k) plan.push_back({j, std::min(chunk, j1 - j), k % nslots});
    // Folds (k_accumulate: the chunks' samples into the running per-pixel
    // sums, chunks in sample order) run on the chunk's own slot stream right
    // after the chunk; a fold whose predecessor ran on the other slot first
    // waits for that fold's event.  (A separate accumulation stream shared a
    // hardware queue with slot 0's stream - HIP maps five streams onto
    // GPU_MAX_HW_QUEUES = 4 queues - so a fold waiting for slot 1's chunk
    // blocked slot 0's next launches behind it: profiles/r06c_timeline/.)
    // A slot's next chunk then reuses its samples buffer after its fold in
    // stream order, with no event at all.
    uint32_t prev_slot = 0xFFFFFFFFu;
    auto fold = [&](const Piece& pf) -> int {
        ptg_context::Slot& sl = slots[pf.slot];
        const int first = pf.j == j0, last = pf.j + pf.n >= j1;
        const hipStream_t as = sl.main;
        if(nslots > 1 && prev_slot != 0xFFFFFFFFu && prev_slot != pf.slot)
            PTG_HIP(hipStreamWaitEvent(as, slots[prev_slot].ev_acc, 0));
        if(int r = timed_begin(ctx, K_ACCUM, as)) return r;
        hipLaunchKernelGGL(k_accumulate, dim3(grid_for(pm.npix)), dim3(kBlock), 0, as, pm, pf.n,
                           sl.samples->as<float4>(), ctx->acc.as<float4>(), first, last, (float)cfg->samples_per_pixel,
                           reinterpret_cast<float4*>(out_accum), reinterpret_cast<uchar4*>(out_bgra));
        PTG_HIP(hipGetLastError());
        if(int r = timed_end(ctx, as)) return r;
        if(nslots > 1) PTG_HIP(hipEventRecord(sl.ev_acc, as));
        prev_slot = pf.slot;
        return PTG_OK;
    };
    for(const Piece& pc: plan)
    {
        const uint32_t j = pc.j, nj = pc.n, si = pc.slot;
        ptg_context::Slot& sl = slots[si];
        SlotState& sst = st[si];
        const DevScene sc_ext = walk_scene(si, 0), sc_sh = walk_scene(si, 1);
        PathSoA* S = sst.S;
        TraceOut* trs = sst.trs;
        uint32_t** lists = sst.lists;
        uint32_t* hit_list = sst.hit_list;
        uint32_t* sky_list = sst.sky_list;
        uint32_t* counts = sst.counts;
        const hipStream_t ms = sl.main;
        const size_t lanes = size_t((pm.npix + 7) / 8) * ((nj + 7) / 8) * 64;
        float4* out = sl.samples->as<float4>();
        if(!wf)
        {
            if(int r = timed_begin(ctx, K_MEGA, ms)) return r;
            if(ctx->counting)
                hipLaunchKernelGGL(k_trace<true>, dim3(grid_for(lanes)), dim3(kBlock), 0, ms, sc, pm, j, nj, out,
                                   cnt_for(K_MEGA));
            else
                hipLaunchKernelGGL(k_trace<false>, dim3(grid_for(lanes)), dim3(kBlock), 0, ms, sc, pm, j, nj, out,
                                   nullptr);
            PTG_HIP(hipGetLastError());
            if(int r = timed_end(ctx, ms)) return r;
        }
        else
        {
            PTG_HIP(hipMemsetAsync(counts, 0, kCountWords(rounds) * sizeof(uint32_t), ms));
            const dim3 grid(std::max<uint32_t>(1, std::min<uint32_t>(persistent, grid_for(lanes))));
            if(int r = timed_begin(ctx, K_CAMERA, ms)) return r;
            if(ctx->counting)
                hipLaunchKernelGGL(k_wf_camera<true>, grid, dim3(kBlock), 0, ms, sc, pm, j, nj, uint32_t(lanes),
                                   S[0], counts, out, cnt_for(K_CAMERA));
            else
                hipLaunchKernelGGL(k_wf_camera<false>, grid, dim3(kBlock), 0, ms, sc, pm, j, nj, uint32_t(lanes),
                                   S[0], counts, out, nullptr);
            PTG_HIP(hipGetLastError());
            if(int r = timed_end(ctx, ms)) return r;
            for(uint32_t r = 0; r < rounds; ++r)
            {
                const PathSoA& cur = S[r & 1];
                const PathSoA& nxt = S[(r + 1) & 1];
                const TraceOut& tr = trs[r & 1];
                if(int e = timed_begin(ctx, K_EXTEND, ms)) return e;
                if(ctx->counting)
                    hipLaunchKernelGGL((k_wf_walk<false, true>), ctx->walk_grid[0], dim3(kBlock), ctx->walk_lds[0], ms, sc_ext,
                                       cur, counts, r, nullptr, tr, ctx->walk_xcds[0], cnt_for(K_EXTEND), ws_for(false));
                else
                    hipLaunchKernelGGL((k_wf_walk<false, false>), ctx->walk_grid[0], dim3(kBlock), ctx->walk_lds[0], ms, sc_ext,
                                       cur, counts, r, nullptr, tr, ctx->walk_xcds[0], nullptr, nullptr);
                PTG_HIP(hipGetLastError());
                if(int e = timed_end(ctx, ms)) return e;
                // second stream: the previous round's sky kernel, then this round's
                // shadow walk (independent of the closest-hit walk it runs beside)
                const hipStream_t ss = overlap ? sl.side : ms;
                if(r > 0)
                {
                    if(int e = timed_begin(ctx, K_SHADOW, ss)) return e;
                    if(ctx->counting)
                        hipLaunchKernelGGL((k_wf_walk<true, true>), ctx->walk_grid[1], dim3(kBlock), ctx->walk_lds[1], ss,
                                           sc_sh, cur, counts, r, lists[r & 1], tr, ctx->walk_xcds[1], cnt_for(K_SHADOW),
                                           ws_for(true));
                    else
                        hipLaunchKernelGGL((k_wf_walk<true, false>), ctx->walk_grid[1], dim3(kBlock), ctx->walk_lds[1], ss,
                                           sc_sh, cur, counts, r, lists[r & 1], tr, ctx->walk_xcds[1], nullptr, nullptr);
                    PTG_HIP(hipGetLastError());
                    if(int e = timed_end(ctx, ss)) return e;
                }
                uint32_t* lc = counts + 2 * (rounds + 2) + 2 * r;   // this round's hit / sky list lengths
                uint32_t* rc = counts + 4 * (rounds + 2) + 2 * r;   // this round's redo list lengths (hit, sky)
                // classify/shade need the shadow results, the lists the previous sky
                // kernel read, and the state set it read
                if(overlap)
                {
                    PTG_HIP(hipEventRecord(sl.ev_side, sl.side));
                    PTG_HIP(hipStreamWaitEvent(ms, sl.ev_side, 0));
                }
                if(int e = timed_begin(ctx, K_CLASSIFY, ms)) return e;
                hipLaunchKernelGGL(k_wf_classify, grid, dim3(kBlock), 0, ms, counts, r, tr, hit_list, sky_list, lc);
                PTG_HIP(hipGetLastError());
                if(int e = timed_end(ctx, ms)) return e;
                if(int e = timed_begin(ctx, K_SHADE, ms)) return e;
                // the certified pass, then the exact pass over the paths it listed
                if(ctx->counting)
                    hipLaunchKernelGGL((k_wf_shade<true, ShadeMath>), grid, dim3(kBlock), 0, ms, sc, cur, nxt, counts, r, tr,
                                       hit_list, lc, lists[(r + 1) & 1], trs[(r + 1) & 1].shadow, out, sst.redo_hit, rc,
                                       cnt_for(K_SHADE), redo_tally);
                else
                    hipLaunchKernelGGL((k_wf_shade<false, ShadeMath>), grid, dim3(kBlock), 0, ms, sc, cur, nxt, counts, r,
                                       tr, hit_list, lc, lists[(r + 1) & 1], trs[(r + 1) & 1].shadow, out, sst.redo_hit,
                                       rc, nullptr, nullptr);
                if constexpr(ShadeMath::kFast)
                {
                    if(ctx->counting)
                        hipLaunchKernelGGL((k_wf_shade<true, MathExact>), dim3(kRedoGrid), dim3(kBlock), 0, ms, sc, cur,
                                           nxt, counts, r, tr, sst.redo_hit, rc, lists[(r + 1) & 1],
                                           trs[(r + 1) & 1].shadow, out, nullptr, nullptr, cnt_for(K_SHADE), nullptr);
                    else
                        hipLaunchKernelGGL((k_wf_shade<false, MathExact>), dim3(kRedoGrid), dim3(kBlock), 0, ms, sc, cur,
                                           nxt, counts, r, tr, sst.redo_hit, rc, lists[(r + 1) & 1],
                                           trs[(r + 1) & 1].shadow, out, nullptr, nullptr, nullptr, nullptr);
                }
                PTG_HIP(hipGetLastError());
                if(int e = timed_end(ctx, ms)) return e;
                // escaped rays retire without feeding the next round: their
                // double-precision atmosphere runs on the second stream, overlapping
                // the next round's latency-bound walks (started beside shade instead,
                // the two compete for registers: 9% slower on frame 0)
                if(overlap)
                {
                    PTG_HIP(hipEventRecord(sl.ev_main, ms));
                    PTG_HIP(hipStreamWaitEvent(sl.side, sl.ev_main, 0));
                }
                if(int e = timed_begin(ctx, K_SKY, ss)) return e;
                if(ctx->counting)
                    hipLaunchKernelGGL(k_wf_sky<true>, grid, dim3(kBlock), 0, ss, sc, cur, tr, r, sky_list, lc, out,
                                       cnt_for(K_SHADE));
                else
                    hipLaunchKernelGGL(k_wf_sky<false>, grid, dim3(kBlock), 0, ss, sc, cur, tr, r, sky_list, lc, out, nullptr);
                PTG_HIP(hipGetLastError());
                if(int e = timed_end(ctx, ss)) return e;
            }
            if(overlap)
            {   // join before accumulate
                PTG_HIP(hipEventRecord(sl.ev_side, sl.side));
                PTG_HIP(hipStreamWaitEvent(ms, sl.ev_side, 0));
            }
        }
        if(int r = fold(pc)) return r;
    }
    if(nslots > 1 && prev_slot != 0xFFFFFFFFu && slots[prev_slot].main != ctx->stream)
        PTG_HIP(hipStreamWaitEvent(ctx->stream, slots[prev_slot].ev_acc, 0));   // the caller's stream sees the whole render
#if PTG_DEBUG
    {
        uint32_t dbg[kDebugSlots];
        PTG_HIP(hipStreamSynchronize(ctx->stream));
        PTG_HIP(hipMemcpy(dbg, ctx->debug.p, sizeof(dbg), hipMemcpyDeviceToHost));
        std::string bad;
        static const char* names[kDebugSlots] = {"node record", "triangle", "instance", "NEE list", "shade list", "walk stack", "", ""};
        for(uint32_t k = 0; k < kDebugSlots; ++k)
            if(dbg[k]) bad += std::string(bad.empty() ? "" : ", ") + names[k] + " index out of range x" + std::to_string(dbg[k]);
        if(!bad.empty())
        {
            PTG_HIP(hipMemset(ctx->debug.p, 0, sizeof(dbg)));
            return fail(PTG_E_RANGE, "PTG_DEBUG: " + bad);
        }
    }
#endif
    if(ctx->counting)
    {
        unsigned long long host[kCounterWords];
        PTG_HIP(hipMemcpyAsync(host, ctx->counters.p, sizeof(host), hipMemcpyDeviceToHost, ctx->stream));
        PTG_HIP(hipStreamSynchronize(ctx->stream));
        for(int k = 0; k < 2 * WS_COUNT; ++k) ctx->walk_stats[k / WS_COUNT][k % WS_COUNT] = host[K_KINDS * 8 + k];
        for(int k = 0; k < kRedoWords; ++k) ctx->redo_stats[k] = host[K_KINDS * 8 + 2 * WS_COUNT + k];
        for(int i = 0; i < 8; ++i)
        {
            ctx->last_counters[i] = 0;
            for(int k = 0; k < K_KINDS; ++k)
            {
                ctx->kind_counters[k][i] = host[k * 8 + i];
                ctx->last_counters[i] += host[k * 8 + i];
            }
        }
    }
    return PTG_OK;
}

int timed_begin(ptg_context* ctx, int kind, hipStream_t st)
{
    if(!ctx->timing) return PTG_OK;
    if(ctx->ev_used == ctx->ev_start.size())
    {
        hipEvent_t a, b;
        PTG_HIP(hipEventCreate(&a));
        PTG_HIP(hipEventCreate(&b));
        ctx->ev_start.push_back(a);
        ctx->ev_stop.push_back(b);
        ctx->ev_kind.push_back(0);
    }
    ctx->ev_kind[ctx->ev_used] = kind;
    PTG_HIP(hipEventRecord(ctx->ev_start[ctx->ev_used], st ? st : ctx->stream));
    return PTG_OK;
}

int timed_end(ptg_context* ctx, hipStream_t st)
{
    if(!ctx->timing) return PTG_OK;
    PTG_HIP(hipEventRecord(ctx->ev_stop[ctx->ev_used++], st ? st : ctx->stream));
    return PTG_OK;
}

} // namespace

extern "C" {

// a launch-geometry knob from the environment (timing experiments only:
// no result depends on it), else its default
static uint32_t env_knob(const char* name, uint32_t dflt)
{
    const char* v = getenv(name);
    if(!v || !*v) return dflt;
    char* end = nullptr;
    const unsigned long x = strtoul(v, &end, 10);
    return (end && *end == 0 && x <= 64) ? uint32_t(x) : dflt;
}

int ptg_context_create(int device, ptg_context** out)
{
    if(!out) return fail(PTG_E_INVALID, "null out");
    *out = nullptr;
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if(e != hipSuccess || n == 0) return fail(PTG_E_NODEVICE, "no HIP device available");
    if(device < 0 || device >= n) return fail(PTG_E_NODEVICE, "device ordinal out of range");
    hipDeviceProp_t prop;
    PTG_HIP(hipGetDeviceProperties(&prop, device));
    if(strncmp(prop.gcnArchName, "gfx950", 6) != 0)
        return fail(PTG_E_NODEVICE, std::string("device is ") + prop.gcnArchName + ", this build targets gfx950");
    std::unique_ptr<ptg_context> ctx(new ptg_context());
    ctx->device = device;
    // grid-stride kernels (camera, classify, shade, sky): 32 blocks per CU,
    // measured best of 3..128
    ctx->persistent_blocks = uint32_t(std::max(1, prop.multiProcessorCount)) * 32u;
    // timing knobs: chunk size and HBM share of a renderer that owns the GPU
    ctx->chunk_log2 = std::min<uint32_t>(28u, std::max<uint32_t>(16u, env_knob("PTG_CHUNK_LOG2", ctx->chunk_log2)));
    ctx->hbm_pct = std::min<uint32_t>(70u, std::max<uint32_t>(5u, env_knob("PTG_HBM_SHARE", ctx->hbm_pct)));
    // Walk residency: each walk lane holds its world ray (32 B) and its stack
    // window (8 x kCap B) in LDS, so the walk blocks' LDS sets how many are
    // resident per CU: kWalkResident (the LDS is padded to that share).
    const uint32_t lds_cu = prop.maxSharedMemoryPerMultiProcessor ? uint32_t(prop.maxSharedMemoryPerMultiProcessor) : 65536u;
    const uint32_t lds_need[2] = {kBlock * uint32_t(sizeof(WalkCold) + WalkStackOf<false>::type::kLaneBytes),
                                  kBlock * uint32_t(sizeof(WalkCold) + WalkStackOf<true>::type::kLaneBytes)};
    for(int k = 0; k < 2; ++k)
    {
        const uint32_t resident = env_knob(k ? "PTG_WALK_RESIDENT_ANY" : "PTG_WALK_RESIDENT", kWalkResident[k]);
        ctx->walk_lds[k] = std::max<uint32_t>(lds_need[k], resident ? (lds_cu / resident) / 1024u * 1024u : 0u);
    }
    // One wave of walk blocks, 3 per CU although the LDS holds 4: every block
    // is resident from the start (no oversubscription), and the fourth slot's
    // LDS and registers take the other chunk pipeline's shade and sky waves,
    // which cannot sit beside four walk blocks (their LDS fills the CU).
    // Measured at 1024 spp against the round-1 choice (4 x the resident grid):
    // frame 0 464 vs 495 ms, frame 450 2827 vs 2843, frame 1400 2004 vs 2012
    // (profiles/r02o_grid/).
    int per_cu = 0;
    const void* walks[2] = {reinterpret_cast<const void*>(k_wf_walk<false, false>),
                            reinterpret_cast<const void*>(k_wf_walk<true, false>)};
    for(int k = 0; k < 2; ++k)
    {
        per_cu = 0;
        if(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, walks[k], kBlock, ctx->walk_lds[k]) != hipSuccess ||
           per_cu <= 0)
            per_cu = int(kWalkResident[k] ? kWalkResident[k] : 1u);
        const uint32_t blocks = env_knob(k ? "PTG_WALK_BLOCKS_ANY" : "PTG_WALK_BLOCKS", kWalkBlocksPerCu[k]);
        ctx->walk_grid[k] = std::min<uint32_t>(uint32_t(per_cu), std::max(1u, blocks)) * uint32_t(prop.multiProcessorCount);
        ctx->walk_xcds[k] = (ctx->walk_grid[k] % 8 == 0 && kBands % 8 == 0) ? 8u : 1u;
    }
    PTG_HIP(hipSetDevice(device));
#if PTG_DEBUG
    PTG_HIP(ctx->debug.reserve(kDebugSlots * sizeof(uint32_t)));
    PTG_HIP(hipMemset(ctx->debug.p, 0, kDebugSlots * sizeof(uint32_t)));
#endif
    PTG_HIP(hipStreamCreateWithFlags(&ctx->side, hipStreamNonBlocking));
    PTG_HIP(hipEventCreateWithFlags(&ctx->ev_main, hipEventDisableTiming));
    PTG_HIP(hipEventCreateWithFlags(&ctx->ev_side, hipEventDisableTiming));
    for(uint32_t k = 1; k < kWfSlots; ++k)
    {
        ptg_context::Slot& b = ctx->slot[k];
        PTG_HIP(hipStreamCreateWithFlags(&b.main, hipStreamNonBlocking));
        PTG_HIP(hipStreamCreateWithFlags(&b.side, hipStreamNonBlocking));
        PTG_HIP(hipEventCreateWithFlags(&b.ev_main, hipEventDisableTiming));
        PTG_HIP(hipEventCreateWithFlags(&b.ev_side, hipEventDisableTiming));
    }
    for(uint32_t k = 0; k < kWfSlots; ++k)
    {
        PTG_HIP(hipEventCreateWithFlags(&ctx->slot[k].ev_acc, hipEventDisableTiming));
    }
    PTG_HIP(hipEventCreateWithFlags(&ctx->ev_render_start, hipEventDisableTiming));
    ctx->nslots = kWfSlots;
    *out = ctx.release();
    return PTG_OK;
}

void ptg_context_destroy(ptg_context* ctx)
{
    if(!ctx) return;
    (void)hipSetDevice(ctx->device);
    (void)hipDeviceSynchronize();
    delete ctx;
}

int ptg_context_get_stream(ptg_context* ctx, void** out)
{
    if(!ctx || !out) return fail(PTG_E_INVALID, "ptg_context_get_stream: null argument");
    *out = static_cast<void*>(ctx->stream);
    return PTG_OK;
}

int ptg_context_device(ptg_context* ctx, int* out)
{
    if(!ctx || !out) return fail(PTG_E_INVALID, "ptg_context_device: null argument");
    *out = ctx->device;
    return PTG_OK;
}

int ptg_context_set_stream(ptg_context* ctx, void* stream)
{
    if(int r = bind(ctx)) return r;
    hipStream_t next = static_cast<hipStream_t>(stream);
    if(next != ctx->stream)
    {   // work queued on the old stream (a render still reading blocks,
        // inst_trav, tlas_root) comes before anything queued on the new one,
        // e.g. the next frame's upload
        hipEvent_t ev;
        PTG_HIP(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
        hipError_t e = hipEventRecord(ev, ctx->stream);
        if(e == hipSuccess) e = hipStreamWaitEvent(next, ev, 0);
        (void)hipEventDestroy(ev);
        if(e != hipSuccess) return hip_fail(e, "ptg_context_set_stream: ordering the old stream before the new");
    }
    ctx->stream = next;
    return PTG_OK;
}

int ptg_upload_scene(ptg_context* ctx, const ptg_bvh_node* nodes, const ptg_bvh_link* links, size_t node_count,
                     const uint32_t* indices, size_t index_count, const ptg_float3* pos, const ptg_float3* normal,
                     const ptg_float4* albedo, const ptg_float4* material, size_t vertex_count)
{
    if(int r = bind(ctx)) return r;
    if(!nodes || !links || !indices || !pos || !normal || !albedo || !material || node_count == 0 || index_count % 3)
        return fail(PTG_E_INVALID, "ptg_upload_scene: bad arguments");
    if(node_count >= (1u << 28) / 8 || index_count >= (1u << 31) || vertex_count >= (1u << 31))
        return fail(PTG_E_RANGE, "ptg_upload_scene: scene too large for 32-bit indexing");
    ctx->scene_ready = ctx->frame_ready = false;
    ctx->packed_mesh.clear();
    ctx->cache.clear();
    ctx->blas_on_device = 0;
    try
    {   // the BLASes are packed into blocks on the host when an instance first names them
        ctx->host_nodes.assign(nodes, nodes + node_count);
        ctx->host_links.assign(links, links + 8 * node_count);
        ctx->host_indices.assign(indices, indices + index_count);
        ctx->host_pos.assign(pos, pos + vertex_count);
        ctx->leaf_bounds_ok.clear();
    }
    catch(const std::bad_alloc&)
    {
        return fail(PTG_E_NOMEM, "ptg_upload_scene: host copy of the BVH nodes");
    }
    PTG_HIP(ctx->indices.reserve(index_count * 4));
    PTG_HIP(ctx->pos.reserve(vertex_count * 16));
    PTG_HIP(ctx->normal.reserve(vertex_count * 16));
    PTG_HIP(ctx->albedo.reserve(vertex_count * 16));
    PTG_HIP(ctx->material.reserve(vertex_count * 16));
    // the walks address triangle records by 32-bit byte offsets (BlockWalker::leaf_select)
    if(index_count / 3 * sizeof(TriRec) + 128 > 0xFFFFFFFFull)
        return fail(PTG_E_RANGE, "triangle records above 4 GB (" + std::to_string(index_count / 3) + " triangles)");
    // slack: the walk's leaf phase reads a triangle as four 16-byte rows (the
    // 48-byte record and the next 16 bytes)
    PTG_HIP(ctx->tris.reserve(std::max<size_t>(1, index_count / 3) * sizeof(TriRec) + 128));
    PTG_HIP(ctx->tri_shade.reserve(std::max<size_t>(1, index_count / 3) * sizeof(TriShade)));
    hipStream_t s = ctx->stream;
    PTG_HIP(hipMemcpyAsync(ctx->indices.p, indices, index_count * 4, hipMemcpyHostToDevice, s));
    PTG_HIP(hipMemcpyAsync(ctx->pos.p, pos, vertex_count * 16, hipMemcpyHostToDevice, s));
    PTG_HIP(hipMemcpyAsync(ctx->normal.p, normal, vertex_count * 16, hipMemcpyHostToDevice, s));
    PTG_HIP(hipMemcpyAsync(ctx->albedo.p, albedo, vertex_count * 16, hipMemcpyHostToDevice, s));
    PTG_HIP(hipMemcpyAsync(ctx->material.p, material, vertex_count * 16, hipMemcpyHostToDevice, s));
    PTG_HIP(hipStreamSynchronize(s));
    // whether every vertex albedo and material value is finite: the surface
    // pass retires a zero-throughput path at its last bounce only then
    // (last_bounce_moot: the term it skips is att * X with X made of them)
    ctx->attrs_finite = true;
    for(size_t i = 0; i < vertex_count && ctx->attrs_finite; ++i)
        ctx->attrs_finite = std::isfinite(albedo[i].x) && std::isfinite(albedo[i].y) && std::isfinite(albedo[i].z) &&
                            std::isfinite(albedo[i].w) && std::isfinite(material[i].x) && std::isfinite(material[i].y) &&
                            std::isfinite(material[i].z) && std::isfinite(material[i].w);
    ctx->static_nodes = node_count;
    ctx->index_count = index_count;
    ctx->vertex_count = vertex_count;
    ctx->scene_ready = true;
    return PTG_OK;
}

namespace {

// The body of ptg_upload_frame (which adds the C ABI's exception barrier).
int upload_frame(ptg_context* ctx, const ptg_subframe* subframes, size_t subframe_count, const ptg_tlas_instance* instances,
                 size_t instance_count, const ptg_bvh_node* frame_nodes, const ptg_bvh_link* frame_links, size_t first_node,
                 size_t frame_node_count)
{
    ctx->frame_ready = false;
    hipStream_t s = ctx->stream;

    // Validate every handle and pack the BLASes no earlier frame named plus
    // this frame's TLASes (host/block_bvh.cpp, checked there before any
    // kernel can follow a block link).  What this call packs joins the cache
    // only after every upload succeeded: an upload that fails half-way never
    // leaves the cache claiming records that were not written.
    FramePack fp;
    std::string err;
    if(int r = ctx->cache.pack_frame(ctx->host_nodes.data(), ctx->host_links.data(), ctx->static_nodes, ctx->index_count,
                                     ctx->vertex_count, subframes, subframe_count, instances, instance_count, frame_nodes,
                                     frame_links, first_node, frame_node_count, fp, err))
        return fail(r, "ptg_upload_frame: " + err);
    std::vector<InstTrav> it(instance_count);
    std::vector<InstShade> is(instance_count);
    std::vector<MeshJob> mesh_jobs;
    std::unordered_set<uint32_t> new_mesh;
    for(size_t i = 0; i < instance_count; ++i)
    {
        const ptg_tlas_instance& in = instances[i];
        const uint32_t handle[4] = {fp.inst_root[i], in.m.index_offset / 3, 0u, 0u};
        for(int k = 0; k < 4; ++k)
        {
            float w;
            memcpy(&w, &handle[k], 4);
            it[i].row[k] = make_float4(in.inv_transform.r[k].x, in.inv_transform.r[k].y, in.inv_transform.r[k].z, w);
        }
        for(int k = 0; k < 3; ++k)
        {
            is[i].rot[k * 3 + 0] = in.transform.r[k].x;
            is[i].rot[k * 3 + 1] = in.transform.r[k].y;
            is[i].rot[k * 3 + 2] = in.transform.r[k].z;
        }
        is[i].index_offset = in.m.index_offset;
        is[i].base_vertex_offset = in.m.base_vertex_offset;
        std::fill(is[i].pad, is[i].pad + 5, 0u);
        if(!ctx->packed_mesh.count(in.m.index_offset) && new_mesh.insert(in.m.index_offset).second)
            mesh_jobs.push_back(MeshJob{in.m.index_offset, in.m.triangle_count, in.m.base_vertex_offset, 0});
    }

    // Per instance its TLAS leaf box and the subframes whose TLAS holds it
    // (InstBox, the any-hit walk's occluder candidates): read from the
    // reference-layout TLAS nodes (octant 0's links name the leaves).  A static
    // instance is a leaf of every subframe's TLAS with the same box (computed
    // from its transform alone, bvh.cc:259-281); a dynamic one of exactly one.
    // Anything else is never a candidate.
    // A candidate triangle's BLAS leaf box is computed from its vertices: the
    // instance offers triangle candidates (tri_count > 0) only if every leaf
    // box of its BLAS is exactly its triangle's bounds (checked once per pair).
    auto leaf_bounds_ok = [&](const ptg_tlas_instance& in) {
        const auto key = std::make_tuple(in.blas.node_offset, in.m.index_offset, in.m.base_vertex_offset);
        auto it = ctx->leaf_bounds_ok.find(key);
        if(it != ctx->leaf_bounds_ok.end()) return it->second;
        // (host code built by the host compiler with the builder's flags:
        // fmin / fmax with the reference's tie rule, host/block_bvh.cpp)
        const bool ok = leaf_boxes_are_vertex_bounds(
            ctx->host_nodes.data() + in.blas.node_offset, ctx->host_links.data() + size_t(in.blas.node_offset) * 8,
            in.blas.node_count, ctx->host_indices.data(), ctx->host_indices.size(), ctx->host_pos.data(),
            ctx->host_pos.size(), in.m.index_offset, in.m.triangle_count, in.m.base_vertex_offset);
        ctx->leaf_bounds_ok[key] = ok;
        return ok;
    };
    std::vector<InstBox> ib(instance_count);
    {
        // seen: the distinct subframes whose TLAS names the instance; an
        // instance named twice by one TLAS is never a candidate (the
        // reference builder makes no such frame, the public upload could)
        std::vector<uint32_t> seen(instance_count, 0), last_sf(instance_count, 0xFFFFFFFFu);
        for(size_t i = 0; i < instance_count; ++i)
        {
            const uint32_t tris = leaf_bounds_ok(instances[i]) ? instances[i].m.triangle_count : 0u;
            ib[i] = InstBox{{0, 0, 0}, kInstNoCandidate, {0, 0, 0}, tris};
        }
        for(size_t sf = 0; sf < subframe_count; ++sf)
        {
            const ptg_bvh tl = subframes[sf].tlas;   // ranges validated by pack_frame
            const size_t base = size_t(tl.node_offset) - first_node;
            for(uint32_t n = 0; n < tl.node_count; ++n)
            {
                const ptg_bvh_link& l = frame_links[8 * base + n];
                if(!(l.accept & 0x80000000u)) continue;
                const uint32_t i = l.accept & 0x7FFFFFFFu;
                if(i >= instance_count) continue;
                const ptg_bvh_node& nd = frame_nodes[base + n];
                const InstBox b{{nd.min_x, nd.min_y, nd.min_z}, uint32_t(sf), {nd.max_x, nd.max_y, nd.max_z}, ib[i].tri_count};
                if(last_sf[i] == uint32_t(sf))
                {   // twice in this subframe's TLAS
                    ib[i].sub = kInstNoCandidate;
                    seen[i] = 0xFFFFFFFFu;
                    continue;
                }
                last_sf[i] = uint32_t(sf);
                if(seen[i] == 0xFFFFFFFFu) continue;
                if(seen[i]++ == 0) ib[i] = b;
                else if(memcmp(ib[i].lo, b.lo, 12) != 0 || memcmp(ib[i].hi, b.hi, 12) != 0) ib[i].sub = kInstNoCandidate;
            }
        }
        for(size_t i = 0; i < instance_count; ++i)
            if(seen[i] == 0xFFFFFFFFu) ib[i].sub = kInstNoCandidate;
            else if(seen[i] > 1 && ib[i].sub != kInstNoCandidate)
                ib[i].sub = seen[i] == subframe_count ? kInstAllSubframes : kInstNoCandidate;
    }

    // Device copies, asynchronous: everything the frame uploads is gathered
    // into one of two pinned staging buffers and copied on the context's
    // stream, behind the render already queued there - the host returns at
    // once and the next render queues right behind the copies.  A staging
    // buffer is reused only after its copies of two uploads ago completed.
    // Growing a device buffer frees the old one, which an in-flight render
    // may still read: the context's streams are drained first (rare).
    auto grow = [&](DevBuf& b, size_t n) { return ctx->grow(b, n); };
    // blocks = [BLAS blocks][TLAS blocks]; growing the buffer drops the BLAS
    // blocks already there, which are then uploaded again
    const std::vector<BlockCopy>& old_blas = ctx->cache.blas;
    const size_t blas_total = old_blas.size() + fp.new_blas.size();
    const size_t need = (blas_total + fp.tlas.size()) * sizeof(BlockCopy);
    if(need > 0xFFFFFFFFull)   // the walks address blocks by 32-bit byte offsets (BlockWalker::block_rows)
        return fail(PTG_E_RANGE, "block records above 4 GB (" + std::to_string(need) + " B)");
    if(need > ctx->blocks.bytes)
    {
        PTG_HIP(grow(ctx->blocks, need + need / 8));
        ctx->blas_on_device = 0;
    }
    PTG_HIP(grow(ctx->tlas_root, subframe_count * sizeof(uint32_t)));
    PTG_HIP(grow(ctx->inst_trav, instance_count * sizeof(InstTrav)));
    PTG_HIP(grow(ctx->inst_shade, instance_count * sizeof(InstShade)));
    PTG_HIP(grow(ctx->inst_box, instance_count * sizeof(InstBox)));
    PTG_HIP(grow(ctx->subframes, subframe_count * sizeof(ptg_subframe)));
    PTG_HIP(grow(ctx->polygon, subframe_count * kPolyStride * sizeof(float2)));
    if(!mesh_jobs.empty()) PTG_HIP(grow(ctx->jobs, mesh_jobs.size() * sizeof(MeshJob)));
    BlockCopy* dev = ctx->blocks.as<BlockCopy>();
    struct Part { const void* src; size_t n; void* dst; };
    std::vector<Part> parts;
    if(ctx->blas_on_device < old_blas.size())
        parts.push_back({old_blas.data() + ctx->blas_on_device, (old_blas.size() - ctx->blas_on_device) * sizeof(BlockCopy),
                         dev + ctx->blas_on_device});
    parts.push_back({fp.new_blas.data(), fp.new_blas.size() * sizeof(BlockCopy), dev + old_blas.size()});
    parts.push_back({fp.tlas.data(), fp.tlas.size() * sizeof(BlockCopy), dev + blas_total});
    parts.push_back({fp.tlas_root.data(), subframe_count * sizeof(uint32_t), ctx->tlas_root.p});
    parts.push_back({it.data(), instance_count * sizeof(InstTrav), ctx->inst_trav.p});
    parts.push_back({is.data(), instance_count * sizeof(InstShade), ctx->inst_shade.p});
    parts.push_back({ib.data(), instance_count * sizeof(InstBox), ctx->inst_box.p});
    parts.push_back({subframes, subframe_count * sizeof(ptg_subframe), ctx->subframes.p});
    parts.push_back({mesh_jobs.data(), mesh_jobs.size() * sizeof(MeshJob), ctx->jobs.p});
    size_t total = 0;
    for(const Part& q: parts) total += (q.n + 255) & ~size_t(255);
    HostStage& hs = ctx->stage[ctx->stage_next];
    ctx->stage_next ^= 1u;
    PTG_HIP(hs.reserve(total));
    size_t off = 0;
    for(const Part& q: parts)
    {
        if(q.n == 0) continue;
        char* h = static_cast<char*>(hs.p) + off;
        memcpy(h, q.src, q.n);
        PTG_HIP(hipMemcpyAsync(q.dst, h, q.n, hipMemcpyHostToDevice, s));
        off += (q.n + 255) & ~size_t(255);
    }
    PTG_HIP(hipEventRecord(hs.done, s));
    hipLaunchKernelGGL(k_polygon_table, dim3(grid_for(subframe_count * kPolyStride)), dim3(kBlock), 0, s,
                       ctx->subframes.as<uint8_t>(), uint32_t(subframe_count), ctx->polygon.as<float2>());
    PTG_HIP(hipGetLastError());
    if(!mesh_jobs.empty())
    {
        uint32_t maxt = 0;
        for(const MeshJob& j: mesh_jobs) maxt = std::max(maxt, j.triangle_count);
        dim3 grid(std::min<uint32_t>(grid_for(maxt), 4096), uint32_t(mesh_jobs.size()));
        hipLaunchKernelGGL(k_pack_tris, grid, dim3(kBlock), 0, s, ctx->indices.as<uint32_t>(), ctx->pos.as<float4>(),
                           ctx->tris.as<TriRec>(), ctx->jobs.as<MeshJob>(), ctx->normal.as<float4>(),
                           ctx->albedo.as<float4>(), ctx->material.as<float4>(), ctx->tri_shade.as<TriShade>());
        PTG_HIP(hipGetLastError());
    }

    // commit
    ctx->cache.commit(fp);
    ctx->blas_on_device = ctx->cache.blas.size();
    ctx->packed_mesh.insert(new_mesh.begin(), new_mesh.end());
    ctx->block_count = fp.total_blocks();
    ctx->stack_bound = fp.stack_bound();
    ctx->host_tlas_root = fp.tlas_root;
    ctx->subframe_count = subframe_count;
    ctx->instance_count = instance_count;
    ctx->host_subframes.assign(subframes, subframes + subframe_count);
    ctx->frame_ready = true;
    return PTG_OK;
}

} // namespace

int ptg_upload_frame(ptg_context* ctx, const ptg_subframe* subframes, size_t subframe_count,
                     const ptg_tlas_instance* instances, size_t instance_count, const ptg_bvh_node* frame_nodes,
                     const ptg_bvh_link* frame_links, size_t first_node, size_t frame_node_count)
{
    if(int r = bind(ctx)) return r;
    if(!ctx->scene_ready) return fail(PTG_E_INVALID, "ptg_upload_frame: upload the scene first");
    if(!subframes || !subframe_count || !instances || !instance_count || !frame_nodes || !frame_links || !frame_node_count)
        return fail(PTG_E_INVALID, "ptg_upload_frame: bad arguments");
    if(first_node != ctx->static_nodes)
        return fail(PTG_E_INVALID, "ptg_upload_frame: first_node must equal the uploaded static node count");
    if(first_node + frame_node_count >= (1ull << 31)) return fail(PTG_E_RANGE, "ptg_upload_frame: too many nodes");
    try
    {
        return upload_frame(ctx, subframes, subframe_count, instances, instance_count, frame_nodes, frame_links, first_node,
                            frame_node_count);
    }
    catch(const std::bad_alloc&)
    {
        ctx->frame_ready = false;
        return fail(PTG_E_NOMEM, "ptg_upload_frame: host memory");
    }
}

int ptg_upload_from_scene(ptg_context* ctx, const ptg_scene* scene, int include_static)
{
    ptg_scene_view v;
    if(int r = ptg_scene_view_get(scene, &v)) return r;
    if(include_static)
        if(int r = ptg_upload_scene(ctx, v.nodes, v.links, v.static_node_count, v.indices, v.index_count, v.pos, v.normal,
                                    v.albedo, v.material, v.vertex_count))
            return r;
    return ptg_upload_frame(ctx, v.subframes, v.subframe_count, v.instances, v.instance_count, v.nodes + v.static_node_count,
                            v.links + 8 * v.static_node_count, v.static_node_count, v.node_count - v.static_node_count);
}

int ptg_render(ptg_context* ctx, const ptg_render_config* cfg, uint32_t x0, uint32_t y0, uint32_t w, uint32_t h,
               uint32_t sample_begin, uint32_t sample_end, ptg_float4* out_accum, ptg_uchar4* out_bgra)
{
    if(int r = bind(ctx)) return r;
    if(int r = check_cfg(ctx, cfg, sample_end)) return r;
    if(uint64_t(x0) + w > cfg->width || uint64_t(y0) + h > cfg->height) return fail(PTG_E_RANGE, "rectangle outside the image");
    PixelMap pm{};
    pm.tiles = 0;
    pm.x0 = x0; pm.y0 = y0; pm.w = w; pm.h = h;
    pm.img_w = cfg->width; pm.img_h = cfg->height;
    pm.npix = w * h;
    return render_map(ctx, cfg, pm, sample_begin, sample_end, out_accum, out_bgra);
}

static int tile_map(const ptg_render_config* cfg, uint32_t tw, uint32_t th, uint32_t first, uint32_t stride,
                    uint32_t count, PixelMap& pm)
{
    if(tw == 0 || th == 0 || stride == 0) return fail(PTG_E_INVALID, "bad tile geometry");
    const uint32_t tx = (cfg->width + tw - 1) / tw, ty = (cfg->height + th - 1) / th;
    if(count && uint64_t(first) + uint64_t(count - 1) * stride >= uint64_t(tx) * ty)
        return fail(PTG_E_RANGE, "tile index beyond the image");
    if(uint64_t(count) * tw * th >= (1ull << 31)) return fail(PTG_E_RANGE, "too many tile pixels");
    pm = PixelMap{};
    pm.tiles = 1;
    pm.tw = tw; pm.th = th; pm.tiles_x = tx; pm.first = first; pm.stride = stride;
    pm.img_w = cfg->width; pm.img_h = cfg->height;
    pm.npix = count * tw * th;
    return PTG_OK;
}

int ptg_render_tiles(ptg_context* ctx, const ptg_render_config* cfg, uint32_t tile_w, uint32_t tile_h, uint32_t first_tile,
                     uint32_t tile_stride, uint32_t tile_count, ptg_float4* out_accum, ptg_uchar4* out_bgra)
{
    if(int r = bind(ctx)) return r;
    if(int r = check_cfg(ctx, cfg, cfg ? cfg->samples_per_pixel : 0)) return r;
    PixelMap pm;
    if(int r = tile_map(cfg, tile_w, tile_h, first_tile, tile_stride, tile_count, pm)) return r;
    return render_map(ctx, cfg, pm, 0, cfg->samples_per_pixel, out_accum, out_bgra);
}

int ptg_scatter_tiles(ptg_context* ctx, const ptg_render_config* cfg, uint32_t tile_w, uint32_t tile_h,
                      uint32_t first_tile, uint32_t tile_stride, uint32_t tile_count, const ptg_uchar4* tiles,
                      ptg_uchar4* image)
{
    if(int r = bind(ctx)) return r;
    if(!cfg || !tiles || !image) return fail(PTG_E_INVALID, "ptg_scatter_tiles: bad arguments");
    PixelMap pm;
    if(int r = tile_map(cfg, tile_w, tile_h, first_tile, tile_stride, tile_count, pm)) return r;
    if(pm.npix == 0) return PTG_OK;
    hipLaunchKernelGGL(k_scatter_tiles, dim3(grid_for(pm.npix)), dim3(kBlock), 0, ctx->stream, pm,
                       reinterpret_cast<const uchar4*>(tiles), reinterpret_cast<uchar4*>(image));
    PTG_HIP(hipGetLastError());
    return PTG_OK;
}

int ptg_path_trace_samples(ptg_context* ctx, const ptg_render_config* cfg, size_t n, const ptg_uint2* xy,
                           const int32_t* sample_index, ptg_float4* out)
{
    if(int r = bind(ctx)) return r;
    if(int r = check_cfg(ctx, cfg, 0)) return r;
    if(!n) return PTG_OK;
    if(!xy || !sample_index || !out || n >= (1u << 30)) return fail(PTG_E_INVALID, "ptg_path_trace_samples: bad arguments");
    int32_t jmax = 0;
    for(size_t i = 0; i < n; ++i)
    {
        jmax = std::max(jmax, sample_index[i]);
        if(xy[i].x >= cfg->width || xy[i].y >= cfg->height) return fail(PTG_E_RANGE, "pixel outside the image");
    }
    if(uint64_t(jmax) / cfg->samples_per_motion_blur_step >= ctx->subframe_count)
        return fail(PTG_E_RANGE, "sample index beyond the frame's subframes");
    if(ctx->stack_bound >= PrivStack::kCap) return fail(PTG_E_RANGE, "walk stack bound above the per-sample kernel's stack");
    PTG_HIP(ctx->grow(ctx->tmp_a, n * sizeof(uint2)));
    PTG_HIP(ctx->grow(ctx->tmp_b, n * sizeof(int32_t)));
    PTG_HIP(ctx->grow(ctx->tmp_c, n * sizeof(float4)));
    PTG_HIP(hipMemcpyAsync(ctx->tmp_a.p, xy, n * sizeof(uint2), hipMemcpyHostToDevice, ctx->stream));
    PTG_HIP(hipMemcpyAsync(ctx->tmp_b.p, sample_index, n * sizeof(int32_t), hipMemcpyHostToDevice, ctx->stream));
    hipLaunchKernelGGL(k_sample_list, dim3(grid_for(n)), dim3(kBlock), 0, ctx->stream, ctx->scene_args(cfg), uint32_t(n),
                       ctx->tmp_a.as<uint2>(), ctx->tmp_b.as<int32_t>(), ctx->tmp_c.as<float4>());
    PTG_HIP(hipGetLastError());
    PTG_HIP(hipMemcpyAsync(out, ctx->tmp_c.p, n * sizeof(float4), hipMemcpyDeviceToHost, ctx->stream));
    PTG_HIP(hipStreamSynchronize(ctx->stream));
    return PTG_OK;
}

int ptg_tonemap_device(ptg_context* ctx, size_t n, const ptg_float4* color, ptg_uchar4* out)
{
    if(int r = bind(ctx)) return r;
    if(!n) return PTG_OK;
    if(!color || !out || n >= (1u << 31)) return fail(PTG_E_INVALID, "ptg_tonemap_device: bad arguments");
    hipLaunchKernelGGL(k_tonemap, dim3(grid_for(n)), dim3(kBlock), 0, ctx->stream, uint32_t(n),
                       reinterpret_cast<const float4*>(color), reinterpret_cast<uchar4*>(out));
    PTG_HIP(hipGetLastError());
    return PTG_OK;
}

int ptg_tonemap(ptg_context* ctx, size_t n, const ptg_float4* color, ptg_uchar4* out)
{
    if(int r = bind(ctx)) return r;
    if(!n) return PTG_OK;
    if(!color || !out || n >= (1u << 30)) return fail(PTG_E_INVALID, "ptg_tonemap: bad arguments");
    PTG_HIP(ctx->grow(ctx->tmp_c, n * sizeof(float4)));
    PTG_HIP(ctx->grow(ctx->tmp_a, n * sizeof(uchar4)));
    PTG_HIP(hipMemcpyAsync(ctx->tmp_c.p, color, n * sizeof(float4), hipMemcpyHostToDevice, ctx->stream));
    hipLaunchKernelGGL(k_tonemap, dim3(grid_for(n)), dim3(kBlock), 0, ctx->stream, uint32_t(n), ctx->tmp_c.as<float4>(),
                       ctx->tmp_a.as<uchar4>());
    PTG_HIP(hipGetLastError());
    PTG_HIP(hipMemcpyAsync(out, ctx->tmp_a.p, n * sizeof(uchar4), hipMemcpyDeviceToHost, ctx->stream));
    PTG_HIP(hipStreamSynchronize(ctx->stream));
    return PTG_OK;
}

int ptg_trace_rays(ptg_context* ctx, uint32_t subframe, size_t n, const float* rays, uint32_t* hits)
{
    if(int r = bind(ctx)) return r;
    if(!ctx->scene_ready || !ctx->frame_ready) return fail(PTG_E_INVALID, "scene/frame not uploaded");
    if(subframe >= ctx->subframe_count) return fail(PTG_E_RANGE, "subframe out of range");
    if(!n) return PTG_OK;
    if(!rays || !hits || n >= (1u << 28)) return fail(PTG_E_INVALID, "ptg_trace_rays: bad arguments");
    // the walk's one-compare box test takes the float after tmin by +1 on its
    // bits (BlockWalker::node_block), which needs tmin's sign bit clear; the
    // reference's queries use 0 and MIN_RAY_DIST (path_tracer.hh:342, :420)
    for(size_t i = 0; i < n; ++i)
    {
        uint32_t b;
        memcpy(&b, rays + i * 8 + 6, 4);
        if((b & 0x80000000u) && (b & 0x7FFFFFFFu) <= 0x7F800000u)
            return fail(PTG_E_INVALID, "ptg_trace_rays: ray " + std::to_string(i) + " has a negative or -0 tmin (needs tmin >= +0)");
    }
    PTG_HIP(ctx->grow(ctx->tmp_a, n * 32));
    PTG_HIP(ctx->grow(ctx->tmp_b, n * 32));
    PTG_HIP(hipMemcpyAsync(ctx->tmp_a.p, rays, n * 32, hipMemcpyHostToDevice, ctx->stream));
    if(ctx->stack_bound >= PrivStack::kCap) return fail(PTG_E_RANGE, "walk stack bound above the per-ray kernels' stack");
    hipLaunchKernelGGL(k_rays, dim3(grid_for(n)), dim3(kBlock), 0, ctx->stream, ctx->scene_args(nullptr),
                       ctx->host_tlas_root[subframe], uint32_t(n), ctx->tmp_a.as<float>(), ctx->tmp_b.as<uint32_t>());
    PTG_HIP(hipGetLastError());
    PTG_HIP(hipMemcpyAsync(hits, ctx->tmp_b.p, n * 32, hipMemcpyDeviceToHost, ctx->stream));
    PTG_HIP(hipStreamSynchronize(ctx->stream));
    return PTG_OK;
}

int ptg_last_counters(ptg_context* ctx, uint64_t out[8])
{
    if(!ctx || !out) return fail(PTG_E_INVALID, "ptg_last_counters: bad arguments");
    if(!ctx->counting) return fail(PTG_E_INVALID, "counters disabled (ptg_counters_enable)");
    memcpy(out, ctx->last_counters, sizeof(ctx->last_counters));
    return PTG_OK;
}

int ptg_counters_enable(ptg_context* ctx, int enable)
{
    if(!ctx) return fail(PTG_E_INVALID, "null context");
    ctx->counting = enable != 0;
    return PTG_OK;
}

int ptg_timing_enable(ptg_context* ctx, int enable)
{
    if(!ctx) return fail(PTG_E_INVALID, "null context");
    ctx->timing = enable != 0;
    ctx->ev_used = 0;
    return PTG_OK;
}

int ptg_last_kernel_times(ptg_context* ctx, double ms[8], uint32_t launches[8])
{
    if(int r = bind(ctx)) return r;
    if(!ms || !launches) return fail(PTG_E_INVALID, "ptg_last_kernel_times: bad arguments");
    for(int k = 0; k < 8; ++k) { ms[k] = 0; launches[k] = 0; }
    for(size_t i = 0; i < ctx->ev_used; ++i)
    {
        PTG_HIP(hipEventSynchronize(ctx->ev_stop[i]));
        float t = 0;
        PTG_HIP(hipEventElapsedTime(&t, ctx->ev_start[i], ctx->ev_stop[i]));
        ms[ctx->ev_kind[i]] += t;
        launches[ctx->ev_kind[i]] += 1;
    }
    ctx->ev_used = 0;
    return PTG_OK;
}

int ptg_last_kernel_busy(ptg_context* ctx, double busy_ms[8], double ms[8], uint32_t launches[8])
{
    if(int r = bind(ctx)) return r;
    if(!busy_ms || !ms || !launches) return fail(PTG_E_INVALID, "ptg_last_kernel_busy: bad arguments");
    struct Iv { int kind; double s, e; };
    std::vector<Iv> iv;
    iv.reserve(ctx->ev_used);
    for(size_t i = 0; i < ctx->ev_used; ++i)
    {
        PTG_HIP(hipEventSynchronize(ctx->ev_stop[i]));
        float s = 0, e = 0;
        // every launch's interval on one time axis: relative to the first recorded start
        PTG_HIP(hipEventElapsedTime(&s, ctx->ev_start[0], ctx->ev_start[i]));
        PTG_HIP(hipEventElapsedTime(&e, ctx->ev_start[0], ctx->ev_stop[i]));
        iv.push_back(Iv{ctx->ev_kind[i], double(s), double(e)});
    }
    std::sort(iv.begin(), iv.end(), [](const Iv& a, const Iv& b) { return a.s < b.s; });
    for(int k = 0; k < 8; ++k)
    {
        busy_ms[k] = ms[k] = 0;
        launches[k] = 0;
        bool open = false;        // a merged interval [cs, ce] of kind k is open
        double cs = 0, ce = 0;
        for(const Iv& v: iv)
        {
            if(v.kind != k) continue;
            ms[k] += v.e - v.s;
            launches[k] += 1;
            if(!open || v.s > ce)
            {
                if(open) busy_ms[k] += ce - cs;
                cs = v.s;
                ce = v.e;
                open = true;
            }
            else ce = std::max(ce, v.e);
        }
        if(open) busy_ms[k] += ce - cs;
    }
    ctx->ev_used = 0;
    return PTG_OK;
}

int ptg_last_timing(ptg_context* ctx, double* trace_ms, uint32_t* launches)
{
    if(!trace_ms || !launches) return fail(PTG_E_INVALID, "ptg_last_timing: bad arguments");
    double ms[8];
    uint32_t n[8];
    if(int r = ptg_last_kernel_times(ctx, ms, n)) return r;
    *trace_ms = 0;
    *launches = 0;
    for(int k = 0; k < 8; ++k)
        if(k != K_ACCUM) { *trace_ms += ms[k]; *launches += n[k]; }
    return PTG_OK;
}

int ptg_last_kernel_counters(ptg_context* ctx, uint64_t out[6][8])
{
    if(!ctx || !out) return fail(PTG_E_INVALID, "ptg_last_kernel_counters: bad arguments");
    if(!ctx->counting) return fail(PTG_E_INVALID, "counters disabled (ptg_counters_enable)");
    memcpy(out, ctx->kind_counters, sizeof(ctx->kind_counters));
    return PTG_OK;
}

int ptg_last_redo_stats(ptg_context* ctx, uint64_t out[9])
{
    if(!ctx || !out) return fail(PTG_E_INVALID, "ptg_last_redo_stats: bad arguments");
    if(!ctx->counting) return fail(PTG_E_INVALID, "counters disabled (ptg_counters_enable)");
    static_assert(kRedoWords == 9, "ptg.h documents 9 words");
    memcpy(out, ctx->redo_stats, sizeof(ctx->redo_stats));
    return PTG_OK;
}

int ptg_last_walk_stats(ptg_context* ctx, uint64_t out[2][8])
{
    if(!ctx || !out) return fail(PTG_E_INVALID, "ptg_last_walk_stats: bad arguments");
    if(!ctx->counting) return fail(PTG_E_INVALID, "counters disabled (ptg_counters_enable)");
    static_assert(WS_COUNT == 8, "ptg.h documents 8 walk statistics");
    memcpy(out, ctx->walk_stats, sizeof(ctx->walk_stats));
    return PTG_OK;
}

int ptg_set_hbm_share(ptg_context* ctx, int percent)
{
    if(!ctx || percent < 5 || percent > 70) return fail(PTG_E_INVALID, "ptg_set_hbm_share: 5 .. 70 percent");
    ctx->hbm_pct = uint32_t(percent);
    return PTG_OK;
}

int ptg_set_chunk_paths(ptg_context* ctx, int log2_paths)
{
    if(!ctx || log2_paths < 16 || log2_paths > 28) return fail(PTG_E_INVALID, "ptg_set_chunk_paths: 16 .. 28");
    ctx->chunk_log2 = uint32_t(log2_paths);
    return PTG_OK;
}

int ptg_set_concurrency(ptg_context* ctx, int level)
{
    if(!ctx || level < 0 || level > 2) return fail(PTG_E_INVALID, "ptg_set_concurrency: 0, 1 or 2");
    ctx->concurrency = uint32_t(level);
    return PTG_OK;
}

int ptg_set_pipeline(ptg_context* ctx, int pipeline)
{
    if(!ctx || pipeline < 0 || pipeline > 1) return fail(PTG_E_INVALID, "ptg_set_pipeline: 0 = wavefront, 1 = megakernel");
    ctx->pipeline = pipeline;
    return PTG_OK;
}

int ptg_arith_selftest(ptg_context* ctx)
{
    if(int r = bind(ctx)) return r;
    const int m = ptg_device_selftest(ctx->stream);
    if(m < 0) return fail(PTG_E_HIP, std::string("ptg_arith_selftest: ") + hipGetErrorString(hipError_t(-m)));
    return m;
}

int ptg_synchronize(ptg_context* ctx)
{
    if(int r = bind(ctx)) return r;
    PTG_HIP(hipStreamSynchronize(ctx->stream));
    return PTG_OK;
}

int ptg_device_alloc(ptg_context* ctx, size_t bytes, void** out)
{
    if(int r = bind(ctx)) return r;
    if(!out) return fail(PTG_E_INVALID, "null out");
    PTG_HIP(hipMalloc(out, bytes));
    return PTG_OK;
}

int ptg_device_free(ptg_context* ctx, void* p)
{
    if(int r = bind(ctx)) return r;
    PTG_HIP(hipFree(p));
    return PTG_OK;
}

int ptg_memcpy_d2h(ptg_context* ctx, void* dst, const void* src, size_t bytes)
{
    if(int r = bind(ctx)) return r;
    PTG_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, ctx->stream));
    PTG_HIP(hipStreamSynchronize(ctx->stream));
    return PTG_OK;
}

} // extern "C"
