/* ptg_rccl.h - the multi-GPU frame entry for a C/C++ host that owns an RCCL
 * communicator (libptg_rccl.so, linked against libptg.so and ROCm's
 * librccl).
 *
 * Replaces, for one frame cut over N GPUs, the body of the reference's
 * pixel-parallel loop: `#pragma omp parallel for` over the pixels of
 * baseline_render (/root/reference/main.cc:16-17) and the frame loop that
 * calls it (main.cc:74-101).  Each rank renders an interleaved set of
 * tile_w x tile_h tiles (tile t -> rank t % N, the same partition as
 * ptg_render_tiles and the Python TileShard), then ONE ncclGather of the BGRA
 * tiles to rank 0 over xGMI assembles the framebuffer there
 * (ptg_scatter_tiles).  Every pixel's samples are summed in index order on
 * one GPU, so the image is bit-identical to a single-GPU ptg_render.
 *
 * Kept out of libptg.so on purpose: the Python product path (torch) brings
 * its own librccl.so.1, and a process must not load two.  A C++ host links
 * this library beside librccl; Python uses distributed.render_and_gather.
 *
 * Error convention as ptg.h (0 or a negative PTG_E_* code); the message is
 * ptg_rccl_last_error().  An RCCL failure is PTG_E_RCCL.
 */
#ifndef PTG_RCCL_H
#define PTG_RCCL_H

#include "ptg.h"

/* RCCL's communicator, forward-declared (ncclComm_t is `struct ncclComm*`)
 * so that this header pulls in no HIP headers: their vector types (uint4,
 * float3, ...) clash with the reference's own (math.hh:11-37), which a host
 * built from the reference's sources includes. */
struct ncclComm;

#ifdef __cplusplus
extern "C" {
#endif

#define PTG_E_RCCL (-7)   /* an RCCL call failed (message has the ncclResult_t) */

/* Render this rank's tiles of the frame uploaded to `ctx` and gather them to
 * rank 0 of `comm`, which scatters them into `image_bgra` (a DEVICE buffer
 * of width*height uchar4 on rank 0; ignored, may be NULL, on the others).
 * Before rendering, every rank all-gathers a small record of the call (the
 * config's fields, the tile size, the communicator size): if any rank
 * differs, EVERY rank returns PTG_E_INVALID naming the fields, and nothing is
 * rendered or gathered - no rank waits in a gather of other sizes.  All work
 * is queued on the context's stream (ptg_context_get_stream) and the call
 * returns once rank 0's image is assembled (it synchronises that stream).
 * `comm` must span one rank per GPU, each with its own context. */
int ptg_render_gather(ptg_context* ctx, const ptg_render_config* cfg, uint32_t tile_w, uint32_t tile_h,
                      struct ncclComm* comm, ptg_uchar4* image_bgra);

/* Convenience for hosts without MPI: one rank per GPU with the rank layout of
 * torch.distributed.run / mpirun in the environment - RANK, WORLD_SIZE,
 * LOCAL_RANK (defaults 0, 1, 0).  Sets the HIP device to LOCAL_RANK and
 * creates the communicator (ncclCommInitRank).  Rank 0 makes the
 * ncclUniqueId; with WORLD_SIZE > 1 it reaches the other ranks through the
 * file named by PTG_NCCL_ID_FILE (written atomically by rank 0; the others
 * wait up to `timeout_s` seconds for it; give each run a fresh path: a file
 * left by an earlier run would hand out a stale id).  Outputs may be NULL
 * except `out`. */
int ptg_rccl_comm_init_env(struct ncclComm** out, int* rank, int* world, int* local_rank, int timeout_s);

/* ncclCommDestroy. */
int ptg_rccl_comm_destroy(struct ncclComm* comm);

/* Message of the last failed ptg_render_gather on this thread. */
const char* ptg_rccl_last_error(void);

#ifdef __cplusplus
}
#endif
#endif /* PTG_RCCL_H */
