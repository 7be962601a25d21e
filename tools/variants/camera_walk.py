# variant: camera rays generated in the round-0 closest-hit walk's refill
# (VERDICT r05 item 3).  k_wf_walk<false, COUNT, true> takes queue position
# t of round 0, computes its pixel / sample (chunk_coords), the seed and the
# camera ray (camera_ray, path_tracer.hh:655-691, :429-450) and starts the
# walk from registers; it still writes meta / seed / ray_o / ray_d (the
# shading reads them), but the camera kernel and the walk's 48-B read-back
# per path are gone.  counts[0] comes from a kernel argument (block 0 writes
# it for the later kernels of the round).
import sys
p = sys.argv[1] + "/pt_kernels.hip"
s = open(p).read()


def sub(old, new, count=1):
    global s
    assert s.count(old) == count, (old, s.count(old))
    s = s.replace(old, new)


# kernel: template flag + camera arguments
sub("""template<bool ANY, bool COUNT>
__global__ __launch_bounds__(kBlock) PTG_WALK_ATTR void k_wf_walk(DevScene sc, PathSoA S, const uint32_t* __restrict__ counts,
                                                    uint32_t round, const uint32_t* __restrict__ list, TraceOut tr,
                                                    uint32_t nxcd, unsigned long long* __restrict__ counters,
                                                    unsigned long long* __restrict__ wstats)
{""", """struct CamArgs {
    PixelMap pm;
    uint32_t j0, nj, M;
    float4* out;
};
template<bool ANY, bool COUNT, bool CAM = false>
__global__ __launch_bounds__(kBlock) PTG_WALK_ATTR void k_wf_walk(DevScene sc, PathSoA S, uint32_t* __restrict__ counts,
                                                    uint32_t round, const uint32_t* __restrict__ list, TraceOut tr,
                                                    uint32_t nxcd, unsigned long long* __restrict__ counters,
                                                    unsigned long long* __restrict__ wstats, CamArgs cam)
{
    static_assert(!(CAM && ANY), "camera rays start closest-hit walks");""")
sub("""    const uint32_t n = counts[2 * round + (ANY ? 1 : 0)];
    const uint32_t lane = threadIdx.x & 63u;""", """    const uint32_t n = CAM ? cam.M : counts[2 * round + (ANY ? 1 : 0)];
    if(CAM && blockIdx.x == 0 && threadIdx.x == 0) counts[0] = cam.M;
    uint32_t lives = 0;
    const uint32_t lane = threadIdx.x & 63u;""")
sub("""                            // path state streams once through the caches: non-temporal
                            const uint4 m = nt_load(S.meta + q);
                            w.init(m.z, xyz(nt_load(S.ray_o + q)),
                                   ANY ? xyz(nt_load(S.nee_d + q)) : xyz(nt_load(S.ray_d + q)), tmin, tmax);""",
    """                            if constexpr(CAM)
                            {   // k_wf_camera's lane q, started from registers
                                uint32_t p, jj, x = 0, y = 0;
                                chunk_coords(q, cam.nj, p, jj);
                                const bool in_chunk = p < cam.pm.npix && jj < cam.nj;
                                const bool live = in_chunk && cam.pm.pixel(p, x, y);
                                const uint32_t slot = in_chunk ? jj * cam.pm.npix + p : 0xFFFFFFFFu;
                                f3 o = V3(0.f, 0.f, 0.f), d = V3(0.f, 0.f, 1.f);
                                uint32_t root = kBePop;
                                if(!live)
                                {
                                    if(in_chunk) st_out(cam.out + slot, make_float4(0.f, 0.f, 0.f, 0.f));
                                    st_state(S.meta + q, make_uint4(slot, META_DEAD, kBePop, 0u));
                                }
                                else
                                {
                                    const int32_t j = (int32_t)(cam.j0 + jj);
                                    const uint8_t* sf = subframe_of(sc, j);
                                    u4 seed;
                                    camera_ray(sc, sf, x, y, j, seed, o, d);
                                    const uint32_t sb = (uint32_t)(sf - sc.subframes) / SF_STRIDE;
                                    root = sc.tlas_root[sb];
                                    st_state(S.meta + q, make_uint4(slot, meta_pack(0, false, sb), root, 0u));
                                    st_state(S.seed + q, to_uint4(seed));
                                    ++lives;
                                }
                                st_state(S.ray_o + q, make_float4(o.x, o.y, o.z, 0.f));
                                st_state(S.ray_d + q, make_float4(d.x, d.y, d.z, 0.f));
                                w.init(root, o, d, tmin, tmax);
                            }
                            else
                            {
                            // path state streams once through the caches: non-temporal
                            const uint4 m = nt_load(S.meta + q);
                            w.init(m.z, xyz(nt_load(S.ray_o + q)),
                                   ANY ? xyz(nt_load(S.nee_d + q)) : xyz(nt_load(S.ray_d + q)), tmin, tmax);""")
sub("""                            if(ANY) w.try_candidate(sc, occ_inst, occ_prim, meta_sub(m));""",
    """                            if constexpr(ANY) w.try_candidate(sc, occ_inst, occ_prim, meta_sub(m));
                            }""")
sub("""        flush_counters(cnt, counters, 0);
        if(lane == 0)
            for(int k = 0; k < WS_COUNT; ++k)""", """        flush_counters(cnt, counters, lives);
        if(lane == 0)
            for(int k = 0; k < WS_COUNT; ++k)""")

# launches: existing walks pass empty camera arguments
for tail in ("cnt_for(K_EXTEND), ws_for(false));", "cnt_for(K_SHADOW),\n                                           ws_for(true));"):
    sub(tail, tail[:-2] + ", CamArgs{});")
sub("tr, ctx->walk_xcds[0], nullptr, nullptr);", "tr, ctx->walk_xcds[0], nullptr, nullptr, CamArgs{});")
sub("tr, ctx->walk_xcds[1], nullptr, nullptr);", "tr, ctx->walk_xcds[1], nullptr, nullptr, CamArgs{});")

# round 0: no camera kernel; the camera walk instead of the plain one
sub("""            if(int r = timed_begin(ctx, K_CAMERA, ms)) return r;
            if(ctx->counting)
                hipLaunchKernelGGL(k_wf_camera<true>, grid, dim3(kBlock), 0, ms, sc, pm, j, nj, uint32_t(lanes),
                                   S[0], counts, out, cnt_for(K_CAMERA));
            else
                hipLaunchKernelGGL(k_wf_camera<false>, grid, dim3(kBlock), 0, ms, sc, pm, j, nj, uint32_t(lanes),
                                   S[0], counts, out, nullptr);
            PTG_HIP(hipGetLastError());
            if(int r = timed_end(ctx, ms)) return r;
""", """            const CamArgs cam{pm, j, nj, uint32_t(lanes), out};
""")
sub("""                if(ctx->counting)
                    hipLaunchKernelGGL((k_wf_walk<false, true>), ctx->walk_grid[0],""",
    """                if(r == 0 && ctx->counting)
                    hipLaunchKernelGGL((k_wf_walk<false, true, true>), ctx->walk_grid[0], dim3(kBlock), ctx->walk_lds[0], ms,
                                       sc_ext, cur, counts, r, nullptr, tr, ctx->walk_xcds[0], cnt_for(K_EXTEND), ws_for(false),
                                       cam);
                else if(r == 0)
                    hipLaunchKernelGGL((k_wf_walk<false, false, true>), ctx->walk_grid[0], dim3(kBlock), ctx->walk_lds[0], ms,
                                       sc_ext, cur, counts, r, nullptr, tr, ctx->walk_xcds[0], nullptr, nullptr, cam);
                else if(ctx->counting)
                    hipLaunchKernelGGL((k_wf_walk<false, true>), ctx->walk_grid[0],""")
open(p, "w").write(s)
