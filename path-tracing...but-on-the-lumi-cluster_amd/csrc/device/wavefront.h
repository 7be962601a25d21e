// Wavefront execution of path_trace_pixel (path_tracer.hh:637-741).
//
// The megakernel form (path_trace_sample) keeps a whole path in one lane, so
// a wave lives as long as its longest path and the BVH walk runs at the
// occupancy the shading code's registers allow.  Here one sample's path is
// cut at its ray queries into kernels that each run over a compacted queue of
// live paths:
//
//   camera   seed, film jitter, camera ray                          (:655-671)
//   extend   closest-hit BVH walk of every queued ray                (:686, :720)
//   shadow   any-hit walk of every pending NEE ray                   (:606-608)
//   shade    NEE finish of the previous bounce, MIS / throughput /
//            atmosphere of this ray, then NEE setup + BSDF sample of
//            the next bounce, or retire the path                     (:691-737)
//
// Per path the arithmetic, its order and the RNG draws are exactly those of
// path_trace_sample (same helper functions), only the place where each step
// runs changes - the frame result stays bit-identical to the reference.
//
// Path state is kept in queue order (structure of arrays, one 16-byte record
// per field), so every kernel reads and writes it with fully coalesced
// dwordx4 accesses; survivors are appended with one atomic per wave.
#pragma once
#include "path_tracer.h"

namespace ptg {
namespace dm {

// One ping-pong half of the path state.  Index = queue position.
struct PathSoA {
    uint4* meta;      // slot (sample-buffer index), round | NEE-pending << 8 | subframe << 16, TLAS node count, TLAS node offset
    uint4* seed;      // RNG state
    float4* ray_o;    // ray origin (= NEE shadow-ray origin)
    float4* ray_d;    // ray direction
    float4* att;      // throughput xyz, w = path-space regularisation
    float4* contrib;  // contribution xyz, w = bsdf_pdf of the bounce that made this ray
    float4* batt;     // bsdf attenuation of that bounce
    float4* nee_c;    // pending NEE colour xyz, w = MIS pdf
    float4* nee_d;    // pending NEE direction xyz, w = atmosphere jitter
};

// Per-queue-position results of the trace kernels.
struct TraceOut {
    uint4* hit;       // thit bits, instance, mesh-global triangle (BLAS triangle base + primitive), back_face
    float2* bary;     // barycentrics u, v (w = 1 - u - v is recomputed)
    uint32_t* shadow; // 1 = the pending NEE ray is occluded
};

constexpr uint32_t META_DEAD = 0x200u;   // queue entry with no path (outside the chunk / image)
PTG_D uint32_t meta_round(uint4 m) { return m.y & 0xFFu; }
PTG_D bool meta_nee(uint4 m) { return (m.y >> 8) & 1u; }
PTG_D uint32_t meta_sub(uint4 m) { return m.y >> 16; }
PTG_D uint32_t meta_pack(uint32_t round, bool nee, uint32_t sub) { return round | (nee ? 0x100u : 0u) | (sub << 16); }

// Append `active` lanes of the calling wave to a queue; one atomic per wave.
__device__ __forceinline__ uint32_t wave_append(uint32_t* counter, bool active)
{
    const unsigned long long mask = __ballot(active);
    if(mask == 0) return 0;
    const uint32_t lane = threadIdx.x & 63u;
    const int leader = __ffsll((long long)mask) - 1;
    uint32_t base = 0;
    if((int)lane == leader) base = atomicAdd(counter, (uint32_t)__popcll(mask));
    base = __shfl(base, leader);
    return base + (uint32_t)__popcll(mask & ((1ull << lane) - 1ull));
}

struct PathRec {
    uint4 meta, seed;
    f3 ray_o, ray_d, att, contrib, batt;
    float reg, bpdf;
    NeeCandidate nee;
};

PTG_D f3 xyz(float4 v) { return V3(v.x, v.y, v.z); }

// Path state, trace results and per-sample results pass through once per
// round: non-temporal (streaming) accesses, so they do not evict BVH records
// from L2 and the Infinity Cache (measured at 1024 spp: frame 0 -1.3%,
// frame 450 -1.1%).
template<typename T> PTG_D T ld_state(const T* p)
{
    typedef uint32_t v4u __attribute__((ext_vector_type(4)));
    const v4u v = __builtin_nontemporal_load(reinterpret_cast<const v4u*>(p));
    T out;
    __builtin_memcpy(&out, &v, 16);
    return out;
}
template<typename T> PTG_D void st_state(T* p, T value)
{
    typedef uint32_t v4u __attribute__((ext_vector_type(4)));
    v4u v;
    __builtin_memcpy(&v, &value, 16);
    __builtin_nontemporal_store(v, reinterpret_cast<v4u*>(p));
}
// per-sample results (written once by shade / sky / camera, read once by k_accumulate)
template<typename T> PTG_D T ld_out(const T* p) { return ld_state(p); }
template<typename T> PTG_D void st_out(T* p, T value) { st_state(p, value); }

PTG_D void store_path(const PathSoA& S, uint32_t q, const PathRec& p)
{
    st_state(S.meta + q, p.meta);
    st_state(S.seed + q, p.seed);
    st_state(S.ray_o + q, make_float4(p.ray_o.x, p.ray_o.y, p.ray_o.z, 0.f));
    st_state(S.ray_d + q, make_float4(p.ray_d.x, p.ray_d.y, p.ray_d.z, 0.f));
    st_state(S.att + q, make_float4(p.att.x, p.att.y, p.att.z, p.reg));
    st_state(S.contrib + q, make_float4(p.contrib.x, p.contrib.y, p.contrib.z, p.bpdf));
    st_state(S.batt + q, make_float4(p.batt.x, p.batt.y, p.batt.z, 0.f));
    if(!meta_nee(p.meta)) return;   // no pending NEE ray: its records are never read
    st_state(S.nee_c + q, make_float4(p.nee.color.x, p.nee.color.y, p.nee.color.z, p.nee.mis_pdf));
    st_state(S.nee_d + q, make_float4(p.nee.dir.x, p.nee.dir.y, p.nee.dir.z, p.nee.jitter));
}

// `carried` = false for round 0 (camera rays): the camera writes only meta,
// seed and the ray, and shade_path's round-0 branch writes throughput,
// contribution, bounce and NEE fields before it reads them, so those five
// records (80 B per path) are not fetched.
PTG_D PathRec load_path(const PathSoA& S, uint32_t q, bool carried = true)
{
    PathRec p;
    p.meta = ld_state(S.meta + q);
    p.seed = ld_state(S.seed + q);
    const float4 ro = ld_state(S.ray_o + q), rd = ld_state(S.ray_d + q);
    p.ray_o = xyz(ro);
    p.ray_d = xyz(rd);
    if(!carried)
    {
        p.att = p.contrib = p.batt = V3(0, 0, 0);
        p.reg = p.bpdf = 0;
        p.nee = NeeCandidate{V3(0, 0, 0), V3(0, 0, 0), 0, 0};
        return p;
    }
    // the pending NEE candidate is read only by paths that have one (classify
    // groups those paths together, so a wave mostly takes one side)
    float4 nc = make_float4(0.f, 0.f, 0.f, 0.f), nd = nc;
    if(meta_nee(p.meta))
    {
        nc = ld_state(S.nee_c + q);
        nd = ld_state(S.nee_d + q);
    }
    const float4 a = ld_state(S.att + q), c = ld_state(S.contrib + q);
    p.att = xyz(a);
    p.reg = a.w;
    p.contrib = xyz(c);
    p.bpdf = c.w;
    p.batt = xyz(ld_state(S.batt + q));
    p.nee.color = xyz(nc);
    p.nee.mis_pdf = nc.w;
    p.nee.dir = xyz(nd);
    p.nee.jitter = nd.w;
    return p;
}

PTG_D u4 to_u4(uint4 v) { return u4{v.x, v.y, v.z, v.w}; }
PTG_D uint4 to_uint4(u4 v) { return make_uint4(v.x, v.y, v.z, v.w); }

// Shade one queued path after its current ray was traced (and its pending
// NEE ray, if any, tested).  Returns SH_CONTINUE when the path continues (p
// is then its state for the next round), SH_DONE when it retired (its sample
// written), SH_REDO (MathFast only) when a rounding certificate failed:
// nothing was written and the path must be shaded again with MathExact.
//
// KIND as in hit_info: the sky kernel instantiates KIND = 2 (the path's ray
// missed, so the path ends here), the surface kernel KIND = 1.
enum ShadeResult { SH_DONE = 0, SH_CONTINUE = 1, SH_REDO = 2 };
template<bool COUNT, int KIND = 0, class MP = MathExact>
PTG_D ShadeResult shade_path(const DevScene& sc, PathRec& p, const Hit& h, bool occluded, float4* out_samples,
                             Counters& cnt, MP& mp)
{
    if(p.meta.y & META_DEAD) return SH_DONE;
    const uint8_t* sf = sc.subframes + size_t(meta_sub(p.meta)) * SF_STRIDE;
    const Light L = light_of(sf);
    const uint32_t round = meta_round(p.meta);
    u4 seed = to_u4(p.seed);
    if(round > 0)
    {   // end of bounce round-1: its NEE term (it reads nothing of the hit, so
        // it runs before the hit's shading: fewer registers live across it)
        f3 nee = V3(0, 0, 0);
        if(meta_nee(p.meta) && !occluded) nee = nee_finish(p.nee, p.ray_o, mp);
        p.contrib = p.contrib + p.att * nee;
    }
    HitInfo info = hit_info<COUNT, KIND>(sc, L, p.ray_o, p.ray_d, h, cnt);
    if(round == 0)
    {   // primary ray (path_tracer.hh:686-693)
        f3 attenuation, in_scatter;
        atmosphere_scattering(seed, L, p.ray_o, p.ray_d, info.thit, attenuation, in_scatter, mp);
        p.att = attenuation;
        p.contrib = V3(0, 0, 0) + (in_scatter + (attenuation * info.albedo) * info.emission);
        p.reg = 1.0f;
    }
    else   // the bounce ray's tail
        bounce_tail<MP, KIND != 2>(seed, L, p.ray_o, p.ray_d, info, p.batt, p.bpdf, p.att, p.contrib, p.reg, mp);
    if(KIND == 2 || !(round < sc.max_bounces && info.thit > 0))
    {
        if(MP::kFast && mp.fail_mask) return SH_REDO;
        st_out(out_samples + p.meta.x, make_float4(p.contrib.x, p.contrib.y, p.contrib.z, 0.f));
        return SH_DONE;
    }
    // bounce `round` (path_tracer.hh:699-720): NEE setup, BSDF sample, next ray
    const Material M{info.albedo, info.roughness, info.metallic, info.transmission, info.eta};
    const f3 view = tangent_view(p.ray_d, info);
    // a shadow ray whose outcome cannot change the result is not traced: the
    // sun ray is below the ground (nee_shadow_moot), or the path's throughput
    // is zero (nee_term_moot)
#ifndef PTG_ZERO_ATT_MOOT
#define PTG_ZERO_ATT_MOOT 1
#endif
    const bool pending = nee_prepare(seed, L, info, M, view, p.nee, mp) && !nee_shadow_moot(p.nee, info.pos) &&
                         !(PTG_ZERO_ATT_MOOT && nee_term_moot(p.att, p.contrib, p.nee));
    const f4 ub = uniform4(seed);
    f3 tdir, batt;
    float bpdf;
    bsdf_sample(V3(ub.x, ub.y, ub.z), view, M, tdir, batt, bpdf, mp);
    p.ray_d = normalize(mul_m3v3(info.tbn, tdir));
    p.ray_o = info.pos;
    p.batt = batt;
    p.bpdf = bpdf;
    p.seed = to_uint4(seed);
#ifndef PTG_ZERO_ATT_RETIRE
#define PTG_ZERO_ATT_RETIRE 1
#endif
    if(PTG_ZERO_ATT_RETIRE && round + 1 == sc.max_bounces && !pending && sc.attrs_finite &&
       last_bounce_moot(p.att, batt, bpdf, p.contrib, L))
    {   // the last bounce would add +-0 terms only: the contribution is final
        if(MP::kFast && mp.fail_mask) return SH_REDO;
        st_out(out_samples + p.meta.x, make_float4(p.contrib.x, p.contrib.y, p.contrib.z, 0.f));
        return SH_DONE;
    }
    p.meta.y = meta_pack(round + 1, pending, meta_sub(p.meta));
    if(MP::kFast && mp.fail_mask) return SH_REDO;
    return SH_CONTINUE;
}

} // namespace dm
} // namespace ptg
