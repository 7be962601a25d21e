// libptg_rccl.so: ptg_render_gather (include/ptg_rccl.h) - one frame over the
// ranks of an RCCL communicator, assembled on rank 0 by a single ncclGather.
//
// The partition is ptg_render_tiles' interleaved tile set: tile t of the
// ceil(W / tw) x ceil(H / th) grid belongs to rank t % N (interleaving spreads
// the frame's up-to-7x per-pixel cost differences).  Rank r
// renders its count(r) tiles densely into a buffer sized for rank 0's count
// (the largest), so every rank sends the same byte count; rank 0 receives N
// such buffers back to back and scatters each rank's tiles into the image.
// Built on the public C ABI of libptg.so only (render, scatter, stream).
#include "ptg_rccl.h"

#include <hip/hip_runtime_api.h>
#include <rccl/rccl.h>

#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <thread>
#include <vector>

namespace {

thread_local std::string g_err;

int fail(int code, const std::string& msg)
{
    g_err = msg;
    return code;
}

int hip_fail(hipError_t e, const char* what)
{
    return fail(PTG_E_HIP, std::string(what) + ": " + hipGetErrorString(e));
}

int nccl_fail(ncclResult_t e, const char* what)
{
    return fail(PTG_E_RCCL, std::string(what) + ": " + ncclGetErrorString(e));
}

int ptg_fail(int rc, const char* what)
{
    return fail(rc, std::string(what) + ": " + (ptg_last_error() ? ptg_last_error() : "?"));
}

// device buffers freed on every exit path
struct DevBufs {
    std::vector<void*> p;
    ~DevBufs()
    {
        for(void* q : p) (void)hipFree(q);
    }
    hipError_t alloc(void** out, size_t bytes)
    {
        hipError_t e = hipMalloc(out, bytes ? bytes : 1);
        if(e == hipSuccess) p.push_back(*out);
        return e;
    }
};

constexpr int kFields = 10;
const char* const kNames[kFields] = {"abi", "width", "height", "samples_per_pixel", "max_bounces", "student_id",
                                     "samples_per_motion_blur_step", "tile_w", "tile_h", "world"};

} // namespace

extern "C" const char* ptg_rccl_last_error(void)
{
    return g_err.c_str();
}

static int env_int(const char* name, int dflt)
{
    const char* v = getenv(name);
    return (v && *v) ? atoi(v) : dflt;
}

extern "C" int ptg_rccl_comm_init_env(struct ncclComm** out, int* rank_out, int* world_out, int* local_out,
                                      int timeout_s)
{
    if(!out) return fail(PTG_E_INVALID, "ptg_rccl_comm_init_env: null out");
    *out = nullptr;
    const int rank = env_int("RANK", 0), world = env_int("WORLD_SIZE", 1), local = env_int("LOCAL_RANK", 0);
    if(world < 1 || rank < 0 || rank >= world || local < 0)
        return fail(PTG_E_INVALID, "ptg_rccl_comm_init_env: RANK " + std::to_string(rank) + " of WORLD_SIZE " +
                                       std::to_string(world) + ", LOCAL_RANK " + std::to_string(local));
    ncclUniqueId id;
    ncclResult_t ne;
    if(rank == 0 && (ne = ncclGetUniqueId(&id)) != ncclSuccess) return nccl_fail(ne, "ncclGetUniqueId");
    if(world > 1)
    {
        const char* path = getenv("PTG_NCCL_ID_FILE");
        if(!path || !*path)
            return fail(PTG_E_INVALID, "ptg_rccl_comm_init_env: WORLD_SIZE > 1 needs PTG_NCCL_ID_FILE");
        if(rank == 0)
        {
            const std::string tmp = std::string(path) + ".tmp";
            FILE* f = fopen(tmp.c_str(), "wb");
            const bool ok = f && fwrite(&id, sizeof id, 1, f) == 1;
            if(f && fclose(f) != 0) return fail(PTG_E_IO, "ptg_rccl_comm_init_env: writing " + tmp);
            if(!ok || rename(tmp.c_str(), path) != 0) return fail(PTG_E_IO, "ptg_rccl_comm_init_env: writing " + tmp);
        }
        else
        {
            bool got = false;
            const auto t0 = std::chrono::steady_clock::now();
            while(!got)
            {
                if(FILE* f = fopen(path, "rb"))
                {
                    got = fread(&id, sizeof id, 1, f) == 1;
                    fclose(f);
                }
                if(got) break;
                if(std::chrono::steady_clock::now() - t0 > std::chrono::seconds(timeout_s > 0 ? timeout_s : 120))
                    return fail(PTG_E_IO, std::string("ptg_rccl_comm_init_env: no ncclUniqueId in ") + path);
                std::this_thread::sleep_for(std::chrono::milliseconds(50));
            }
        }
    }
    hipError_t he = hipSetDevice(local);
    if(he != hipSuccess) return hip_fail(he, "ptg_rccl_comm_init_env: hipSetDevice(LOCAL_RANK)");
    ncclComm_t comm = nullptr;
    if((ne = ncclCommInitRank(&comm, world, id, rank)) != ncclSuccess) return nccl_fail(ne, "ncclCommInitRank");
    *out = comm;
    if(rank_out) *rank_out = rank;
    if(world_out) *world_out = world;
    if(local_out) *local_out = local;
    return PTG_OK;
}

extern "C" int ptg_rccl_comm_destroy(struct ncclComm* comm)
{
    if(!comm) return fail(PTG_E_INVALID, "ptg_rccl_comm_destroy: null communicator");
    ncclResult_t ne = ncclCommDestroy(comm);
    return ne == ncclSuccess ? PTG_OK : nccl_fail(ne, "ncclCommDestroy");
}

extern "C" int ptg_render_gather(ptg_context* ctx, const ptg_render_config* cfg, uint32_t tile_w, uint32_t tile_h,
                                 struct ncclComm* comm, ptg_uchar4* image_bgra)
{
    if(!ctx || !cfg || !comm) return fail(PTG_E_INVALID, "ptg_render_gather: null argument");
    if(tile_w == 0 || tile_h == 0 || cfg->width == 0 || cfg->height == 0)
        return fail(PTG_E_INVALID, "ptg_render_gather: empty tile or image");
    int rank = 0, world = 0, dev = 0;
    ncclResult_t ne = ncclCommUserRank(comm, &rank);
    if(ne == ncclSuccess) ne = ncclCommCount(comm, &world);
    if(ne != ncclSuccess) return nccl_fail(ne, "ptg_render_gather: communicator rank/size");
    if(int rc = ptg_context_device(ctx, &dev)) return ptg_fail(rc, "ptg_render_gather");
    void* sv = nullptr;
    if(int rc = ptg_context_get_stream(ctx, &sv)) return ptg_fail(rc, "ptg_render_gather");
    hipStream_t st = static_cast<hipStream_t>(sv);
    hipError_t he = hipSetDevice(dev);
    if(he != hipSuccess) return hip_fail(he, "ptg_render_gather: hipSetDevice");
    DevBufs bufs;

    // (1) every rank agrees on the call before anything is rendered
    int64_t mine[kFields] = {1, cfg->width, cfg->height, cfg->samples_per_pixel, cfg->max_bounces, cfg->student_id,
                             cfg->samples_per_motion_blur_step, tile_w, tile_h, world};
    void* d_rec = nullptr;
    if((he = bufs.alloc(&d_rec, sizeof(int64_t) * kFields * (size_t(world) + 1))) != hipSuccess)
        return hip_fail(he, "ptg_render_gather: record buffer");
    int64_t* d_mine = static_cast<int64_t*>(d_rec) + size_t(kFields) * world;
    if((he = hipMemcpyAsync(d_mine, mine, sizeof mine, hipMemcpyHostToDevice, st)) != hipSuccess)
        return hip_fail(he, "ptg_render_gather: record upload");
    if((ne = ncclAllGather(d_mine, d_rec, kFields, ncclInt64, comm, st)) != ncclSuccess)
        return nccl_fail(ne, "ptg_render_gather: agreement all-gather");
    std::vector<int64_t> all(size_t(kFields) * world);
    if((he = hipMemcpyAsync(all.data(), d_rec, sizeof(int64_t) * all.size(), hipMemcpyDeviceToHost, st)) != hipSuccess ||
       (he = hipStreamSynchronize(st)) != hipSuccess)
        return hip_fail(he, "ptg_render_gather: record readback");
    std::string diff;
    for(int f = 0; f < kFields; ++f)
    {
        bool same = true;
        for(int r = 1; r < world; ++r) same = same && all[size_t(r) * kFields + f] == all[f];
        if(same) continue;
        diff += diff.empty() ? "" : "; ";
        diff += kNames[f];
        for(int r = 0; r < world; ++r)
            diff += (r ? ", " : " (") + std::string("rank ") + std::to_string(r) + ": " +
                    std::to_string(all[size_t(r) * kFields + f]);
        diff += ")";
    }
    if(!diff.empty()) return fail(PTG_E_INVALID, "ptg_render_gather: the ranks disagree on " + diff);
    if(rank == 0 && !image_bgra) return fail(PTG_E_INVALID, "ptg_render_gather: rank 0 needs an image buffer");

    // (2) this rank's tiles, densely
    const uint32_t tiles_x = (cfg->width + tile_w - 1) / tile_w, tiles_y = (cfg->height + tile_h - 1) / tile_h;
    const uint64_t total = uint64_t(tiles_x) * tiles_y;
    auto count_for = [&](int r) -> uint32_t {
        return total > uint64_t(r) ? uint32_t((total - uint64_t(r) + uint64_t(world) - 1) / uint64_t(world)) : 0u;
    };
    const size_t per_tile = size_t(tile_w) * tile_h;
    const size_t send_px = size_t(count_for(0)) * per_tile;
    void* d_send = nullptr;
    if((he = bufs.alloc(&d_send, send_px * sizeof(ptg_uchar4))) != hipSuccess)
        return hip_fail(he, "ptg_render_gather: tile buffer");
    if((he = hipMemsetAsync(d_send, 0, send_px * sizeof(ptg_uchar4), st)) != hipSuccess)
        return hip_fail(he, "ptg_render_gather: tile buffer clear");
    if(const uint32_t n = count_for(rank))
        if(int rc = ptg_render_tiles(ctx, cfg, tile_w, tile_h, uint32_t(rank), uint32_t(world), n, nullptr,
                                     static_cast<ptg_uchar4*>(d_send)))
            return ptg_fail(rc, "ptg_render_gather: ptg_render_tiles");

    // (3) one gather of the BGRA tiles to rank 0, then the scatter there
    void* d_recv = nullptr;
    if(rank == 0 && (he = bufs.alloc(&d_recv, send_px * sizeof(ptg_uchar4) * size_t(world))) != hipSuccess)
        return hip_fail(he, "ptg_render_gather: gather buffer");
    if((ne = ncclGather(d_send, d_recv, send_px * sizeof(ptg_uchar4), ncclUint8, 0, comm, st)) != ncclSuccess)
        return nccl_fail(ne, "ptg_render_gather: ncclGather");
    if(rank == 0)
        for(int r = 0; r < world; ++r)
            if(const uint32_t n = count_for(r))
                if(int rc = ptg_scatter_tiles(ctx, cfg, tile_w, tile_h, uint32_t(r), uint32_t(world), n,
                                              static_cast<const ptg_uchar4*>(d_recv) + size_t(r) * send_px,
                                              image_bgra))
                    return ptg_fail(rc, "ptg_render_gather: ptg_scatter_tiles");
    if((he = hipStreamSynchronize(st)) != hipSuccess) return hip_fail(he, "ptg_render_gather: synchronise");
    return PTG_OK;
}
