/* ptg.h - C ABI of the MI355X-native path tracer.
 *
 * Drop-in boundary for the reference's per-pixel hot path
 * (Kalache-abdesattar/Path-Tracing...but-on-the-LUMI-cluster @ v1):
 *   path_trace_pixel  path_tracer.hh:637-741
 *   tonemap_pixel     path_tracer.hh:753-771
 *   baseline_render   main.cc:12-46 (the loop that calls them)
 *   ray_query_*       ray_query.hh:111-290 (BVH traversal underneath)
 *
 * Plain C, plain pointers and sizes.  Every type below reproduces the byte
 * layout of the reference type it names (bvh.hh, mesh.hh, scene.hh, math.hh),
 * so a caller holding the reference's std::vectors passes .data() unchanged.
 * NOTE: ptg_float3 is 16 bytes (OpenCL layout, math.hh:36) - never pass HIP's
 * 12-byte float3.
 *
 * Error convention: every int-returning entry returns PTG_OK (0) or a
 * negative PTG_E_* code; ptg_last_error() gives the message.  Nothing calls
 * exit().  One host thread per context; calls on a context are not reentrant
 * (the reference's functions are pure, main.cc drives them from one thread
 * plus OpenMP workers - ptg_render replaces that whole loop).
 */
#ifndef PTG_H
#define PTG_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
#define PTG_ALIGNAS(n) alignas(n)
extern "C" {
#else
#define PTG_ALIGNAS(n) _Alignas(n)
#endif

#define PTG_ABI_VERSION 1

/* ---- reference-layout types ------------------------------------------- */

/* math.hh:31-37 */
typedef struct { PTG_ALIGNAS(8) uint32_t x; uint32_t y; } ptg_uint2;
typedef struct { PTG_ALIGNAS(16) uint32_t x; uint32_t y, z, w; } ptg_uint4;
typedef struct { PTG_ALIGNAS(16) float x; float y, z; } ptg_float3;       /* 16 B */
typedef struct { PTG_ALIGNAS(16) float x; float y, z, w; } ptg_float4;
typedef struct { PTG_ALIGNAS(4) uint8_t x; uint8_t y, z, w; } ptg_uchar4;
/* math.hh:152-153: row vectors */
typedef struct { ptg_float3 r[3]; } ptg_mat3;                              /* 48 B */
typedef struct { ptg_float4 r[4]; } ptg_mat4;                              /* 64 B */

/* bvh.hh:35-39 */
typedef struct { uint32_t node_count, node_offset; } ptg_bvh;
/* bvh.hh:45-49 */
typedef struct { float min_x, min_y, min_z, max_x, max_y, max_z; } ptg_bvh_node;   /* 24 B */
/* bvh.hh:57-67: accept top bit = leaf, rest = payload */
typedef struct { uint32_t accept, cancel; } ptg_bvh_link;
/* mesh.hh:18-28 */
typedef struct { uint32_t vertex_count, triangle_count, index_offset, base_vertex_offset; } ptg_mesh;
/* bvh.hh:73-79 */
typedef struct { ptg_bvh blas; ptg_mesh m; ptg_mat4 transform; ptg_mat4 inv_transform; } ptg_tlas_instance; /* 160 B */
/* scene.hh:7-17 */
typedef struct {
    ptg_mat3 orientation;
    ptg_float3 position;
    float aspect_ratio;
    float inv_focal_length;
    float focal_distance;
    float aperture_angle;
    int32_t aperture_polygon;
    float aperture_radius;
} ptg_camera;                                                              /* 96 B */
/* scene.hh:19-24 */
typedef struct { ptg_float3 direction; ptg_float3 color; float cos_solid_angle; } ptg_directional_light; /* 48 B */
/* scene.hh:26-34 */
typedef struct { ptg_bvh tlas; ptg_camera cam; ptg_directional_light light; } ptg_subframe; /* 160 B */

/* ---- render configuration ---------------------------------------------
 * The reference bakes these in as macros (config.hh:5-29, and
 * path_tracer.hh:431/656/659/697); here they are runtime values.
 */
typedef struct {
    uint32_t width;                        /* IMAGE_WIDTH */
    uint32_t height;                       /* IMAGE_HEIGHT */
    uint32_t samples_per_pixel;            /* SAMPLES_PER_PIXEL */
    uint32_t max_bounces;                  /* MAX_BOUNCES (4 = TESTING preset) */
    uint32_t student_id;                   /* STUDENT_ID, 4th RNG seed word */
    uint32_t samples_per_motion_blur_step; /* SAMPLES_PER_MOTION_BLUR_STEP (8) */
} ptg_render_config;

/* Fill with the reference's shipped values: 640x360, 256 spp, 4 bounces,
 * student id 152121358, 8 samples per motion-blur step (config.hh:5-29). */
void ptg_render_config_default(ptg_render_config* cfg);

/* ---- errors ------------------------------------------------------------ */
#define PTG_OK 0
#define PTG_E_INVALID (-1)   /* bad argument / state */
#define PTG_E_IO (-2)        /* file could not be read or written */
#define PTG_E_NOMEM (-3)     /* host or device allocation failed */
#define PTG_E_HIP (-4)       /* HIP runtime error (message has the hipError_t) */
#define PTG_E_NODEVICE (-5)  /* no usable gfx950 device */
#define PTG_E_RANGE (-6)     /* index / size out of the supported range */

int ptg_abi_version(void);
/* Message of the last error raised on this host thread ("" if none). */
const char* ptg_last_error(void);
/* Host worker threads each of this process's pools (scene load, per-frame
 * TLAS builds, TLAS block packing) may use; 0 (default) = automatic: the CPUs
 * the process may run on (affinity, cgroup CPU quota) divided by the ranks of
 * the node (LOCAL_WORLD_SIZE).  Returns the value now in effect. */
int ptg_set_host_threads(int threads);

/* ---- host-side scene (restatement of scene.cc / bvh.cc / mesh.cc) -------
 * Produces exactly the arrays the reference's load_scene (scene.cc:135) and
 * setup_animation_frame (scene.cc:271) produce, in reference layout.
 */
typedef struct ptg_scene ptg_scene;

typedef struct {
    const ptg_bvh_node* nodes; size_t node_count;     /* bvh_buffers.nodes */
    const ptg_bvh_link* links;                        /* 8 * node_count entries */
    size_t static_node_count;                         /* nodes owned by BLASes (uploaded once) */
    const uint32_t* indices; size_t index_count;      /* mesh_buffers.indices */
    const ptg_float3* pos;                            /* mesh_buffers.pos, vertex_count entries */
    const ptg_float3* normal;
    const ptg_float4* albedo;
    const ptg_float4* material;
    size_t vertex_count;
    const ptg_tlas_instance* instances; size_t instance_count;
    size_t static_instance_count;
    const ptg_subframe* subframes; size_t subframe_count;
} ptg_scene_view;

/* load_scene(): assets_dir must contain data/<name>.obj|.mtl.  The scene
 * depends on the configuration through width/height (camera aspect,
 * scene.cc:284) and samples_per_pixel (subframe count, scene.cc:648-650). */
int ptg_scene_load(const char* assets_dir, const ptg_render_config* cfg, ptg_scene** out);
/* setup_animation_frame() */
int ptg_scene_setup_frame(ptg_scene* s, uint32_t frame_index);
/* Pointers stay valid until the next setup_frame/destroy. */
int ptg_scene_view_get(const ptg_scene* s, ptg_scene_view* out);
/* get_animation_frame_count() (scene.cc:720-724) */
uint32_t ptg_scene_frame_count(const ptg_scene* s);
/* BLAS handle of a named mesh (the scene.meshes map, scene.hh:52); -1 if absent */
int ptg_scene_mesh(const ptg_scene* s, const char* name, ptg_mesh* mesh, ptg_bvh* blas);
void ptg_scene_destroy(ptg_scene* s);

/* write_bmp (bmp.cc:7-63): 24-bit bottom-up BMP from bytes 0..2 of each
 * `stride`-byte pixel of a `pitch`-byte row (BGRA input -> BGR file). */
int ptg_write_bmp(const char* path, uint32_t w, uint32_t h, uint32_t stride, uint32_t pitch,
                  const uint8_t* color_data);

/* ---- GPU renderer -------------------------------------------------------- */
typedef struct ptg_context ptg_context;

/* One context per GPU (device ordinal as seen by HIP).  Fails loudly with
 * PTG_E_NODEVICE if the device is not a gfx950 part. */
int ptg_context_create(int device, ptg_context** out);
void ptg_context_destroy(ptg_context* ctx);
/* hipStream_t the context launches on (NULL = legacy default stream).  Work
 * already queued on the previous stream is ordered before anything queued on
 * the new one (an event recorded there, waited on by the new stream). */
int ptg_context_set_stream(ptg_context* ctx, void* hip_stream);
/* The hipStream_t the context launches on (*out; NULL = the legacy default
 * stream), so a caller can order its own work - e.g. an RCCL collective over
 * the rendered tiles (include/ptg_rccl.h) - after the context's. */
int ptg_context_get_stream(ptg_context* ctx, void** out);
/* The HIP device ordinal of the context (*out). */
int ptg_context_device(ptg_context* ctx, int* out);

/* Once per run: the static part of the arrays (everything load_scene
 * produced).  nodes/links hold node_count BVH nodes (links: 8 per node, the
 * bvh_buffers layout, bvh.cc:218-225).  Host pointers. */
int ptg_upload_scene(ptg_context* ctx,
                     const ptg_bvh_node* nodes, const ptg_bvh_link* links, size_t node_count,
                     const uint32_t* indices, size_t index_count,
                     const ptg_float3* pos, const ptg_float3* normal,
                     const ptg_float4* albedo, const ptg_float4* material, size_t vertex_count);

/* Once per frame: what setup_animation_frame changed.  frame_nodes/links are
 * the TLAS nodes appended after the static ones (node indices
 * first_node .. first_node+frame_node_count-1 of the reference's
 * bvh_buffers; first_node must equal the static node count).  instances is
 * the full instance array (static + this frame's dynamic ones).  Host
 * pointers, read before the call returns (the caller may overwrite them at
 * once); the device copies are queued on the context's stream behind any
 * render already queued there.  The call waits only for the copies of the
 * upload two calls back (its pinned staging is reused) or, when a device
 * buffer must grow, for the stream to drain. */
int ptg_upload_frame(ptg_context* ctx,
                     const ptg_subframe* subframes, size_t subframe_count,
                     const ptg_tlas_instance* instances, size_t instance_count,
                     const ptg_bvh_node* frame_nodes, const ptg_bvh_link* frame_links,
                     size_t first_node, size_t frame_node_count);

/* Convenience: upload_scene + upload_frame from a ptg_scene. */
int ptg_upload_from_scene(ptg_context* ctx, const ptg_scene* s, int include_static);

/* baseline_render() body for a rectangle of the image: for each pixel, sum
 * path_trace_pixel over sample indices [sample_begin, sample_end) in index
 * order in float32 (main.cc:24-39), divide by cfg->samples_per_pixel
 * (main.cc:42) and tonemap (main.cc:43).
 * out_accum (optional, DEVICE pointer, [h][w] ptg_float4): the averaged radiance.
 * out_bgra  (optional, DEVICE pointer, [h][w] ptg_uchar4): tonemap_pixel output.
 * Pixel (x0+i, y0+k) lands at row k, column i.  Asynchronous on the context's
 * stream. */
int ptg_render(ptg_context* ctx, const ptg_render_config* cfg,
               uint32_t x0, uint32_t y0, uint32_t w, uint32_t h,
               uint32_t sample_begin, uint32_t sample_end,
               ptg_float4* out_accum, ptg_uchar4* out_bgra);

/* Same for an interleaved set of tiles (multi-GPU sharding): tiles of
 * tile_w x tile_h pixels numbered row-major over the image; this call renders
 * tiles first_tile, first_tile + tile_stride, ... (tile_count of them) and
 * writes them densely, tile after tile, each tile row-major
 * (tile_w*tile_h pixels per tile; pixels outside the image are left 0). */
int ptg_render_tiles(ptg_context* ctx, const ptg_render_config* cfg,
                     uint32_t tile_w, uint32_t tile_h,
                     uint32_t first_tile, uint32_t tile_stride, uint32_t tile_count,
                     ptg_float4* out_accum, ptg_uchar4* out_bgra);

/* Scatter densely packed tiles (as written by ptg_render_tiles for one
 * first_tile/tile_stride set) into a full image; DEVICE pointers. */
int ptg_scatter_tiles(ptg_context* ctx, const ptg_render_config* cfg,
                      uint32_t tile_w, uint32_t tile_h,
                      uint32_t first_tile, uint32_t tile_stride, uint32_t tile_count,
                      const ptg_uchar4* tiles_bgra, ptg_uchar4* image_bgra);

/* path_trace_pixel (path_tracer.hh:637) for a batch of (pixel, sample_index)
 * pairs: out[i] = path_trace_pixel(xy[i], sample_index[i], ...) (w = 0).
 * HOST pointers; synchronous.  Used for per-sample parity. */
int ptg_path_trace_samples(ptg_context* ctx, const ptg_render_config* cfg, size_t n,
                           const ptg_uint2* xy, const int32_t* sample_index, ptg_float4* out);

/* tonemap_pixel (path_tracer.hh:753) on n colours. HOST pointers; synchronous. */
int ptg_tonemap(ptg_context* ctx, size_t n, const ptg_float4* color, ptg_uchar4* out);
/* The same on DEVICE pointers, asynchronous on the context's stream (the
 * sample-range shard tonemaps the reduced radiance with it). */
int ptg_tonemap_device(ptg_context* ctx, size_t n, const ptg_float4* color, ptg_uchar4* out);

/* Ray-level query through the uploaded scene with subframe `subframe`'s TLAS:
 * rays are 8 floats (origin.xyz, dir.xyz, tmin, tmax).  For each ray, hits
 * gets 8 words {bary.x, bary.y, bary.z, thit (f32), instance_id, primitive_id,
 * back_face, shadowed}: the closest hit of ray_query_proceed/confirm
 * (ray_query.hh:248-290) and the any-hit bool of a single proceed
 * (path_tracer.hh:415-427).  HOST pointers; synchronous.
 * Contract: every tmin is +0 or positive (or NaN / +inf, which no hit
 * passes), as the reference's queries are (0 and MIN_RAY_DIST); a ray with a
 * negative or -0 tmin is refused (PTG_E_INVALID, nothing traced).  Any tmax
 * is accepted. */
int ptg_trace_rays(ptg_context* ctx, uint32_t subframe, size_t n, const float* rays, uint32_t* hits);

/* Work counters of the last ptg_render* call (filled only while counting is
 * on, ptg_counters_enable; counting uses a separate, slower build of the
 * kernels):
 * [0] samples, [1] node visits, [2] triangle tests, [3] BLAS entries,
 * [4] ray queries, [5] closest-hit shades, [6] TLAS node visits (part of [1]),
 * [7] walk-loop iterations of whole waves (diagnostics).  [5] counts shading
 * passes: a surface path the certified pass lists for the exact pass
 * (ptg_last_redo_stats out[0]) is counted twice. */
int ptg_counters_enable(ptg_context* ctx, int enable);
int ptg_last_counters(ptg_context* ctx, uint64_t out[8]);
/* Counters split by kernel kind (same kinds as ptg_last_kernel_times). */
int ptg_last_kernel_counters(ptg_context* ctx, uint64_t out[6][8]);
/* Wavefront walk statistics of the last counted ptg_render* call, for the
 * closest-hit walk (out[0]) and the any-hit walk (out[1]):
 * [0] node phases that loaded block rows (wave instructions of one row),
 * [1] lanes those phases served, [2] leaf phases that loaded a triangle or
 * instance record, [3] lanes they served, [4] refills that started rays,
 * [5] lanes they started, [6] walk-loop iterations, [7] lanes active in them.
 * A node phase issues 7 row loads and a leaf phase 4, each a wave
 * instruction whatever its EXEC mask: [1]/[0] and [3]/[2] are the lanes per
 * vector-memory instruction of the walk. */
int ptg_last_walk_stats(ptg_context* ctx, uint64_t out[2][8]);

/* The certified shading of the last ptg_render* call (counting builds, as
 * ptg_last_counters).  The wavefront pipeline's surface kernel evaluates
 * the path's double-precision exp / pow / sin / cos with the GPU library and
 * proves per evaluation that the float the path keeps is the one glibc's
 * double gives (device/ref_math.h, float_certain); a path with an evaluation
 * the proof does not cover is shaded again with the restated glibc
 * algorithms.  The sky kernel runs the restated glibc algorithms directly
 * and certifies nothing.  out[0]: surface paths shaded again; out[1]:
 * reserved (always 0); out[2..8]: per certificate site (acc_exp, exp_times, add_mul_pow,
 * div_mul_pow, times_cos, times_sin, times_one_minus_div_pow) the paths in
 * which it failed. */
int ptg_last_redo_stats(ptg_context* ctx, uint64_t out[9]);

/* The arithmetic environment the bit-exact results rest on: the known-answer
 * checks of ptg_device.h's ptg_device_selftest, compiled with this library's
 * own flags and run on the context's device, against this host's libm.
 * Returns the mask of failed checks (0: all passed; see ptg_device.h for the
 * bits: FP contraction, glibc exp / pow / sin / cos, tonemap, fmin's tie rule,
 * division), or a negative error code.  A nonzero mask means this host's
 * reference build would not give the bits the GPU gives (a libm other than
 * glibc 2.35's FMA variants), or the library was built with the wrong flags. */
int ptg_arith_selftest(ptg_context* ctx);

/* Per-launch device timing, measured with HIP events recorded around every
 * kernel launch on the context's stream.  Enabling (re)starts the record;
 * every ptg_render* call after that appends its launches, without blocking
 * the host, so host work (e.g. the next frame's setup) keeps overlapping the
 * GPU.  Reading the record (ptg_last_timing / ptg_last_kernel_times) waits
 * for the recorded launches, returns their summed device time and count, and
 * clears it.  ptg_last_timing sums all path-tracing kernels (all kinds but
 * accumulate). */
int ptg_timing_enable(ptg_context* ctx, int enable);
int ptg_last_timing(ptg_context* ctx, double* trace_ms, uint32_t* launches);
/* The same per kernel kind: [0] megakernel, [1] extend (closest-hit walk),
 * [2] shadow (any-hit walk), [3] shade (surface hits), [4] camera,
 * [5] accumulate, [6] sky (rays that left the scene), [7] classify. */
int ptg_last_kernel_times(ptg_context* ctx, double ms[8], uint32_t launches[8]);
/* The same record read as busy time: per kind, the UNION of the recorded
 * launches' [start, end) intervals on one device time axis (busy_ms), beside
 * their plain sum (ms) and count.  Launches of one kind that overlap (the two
 * chunk pipelines) are counted once, so busy_ms never exceeds the wall time
 * of the recorded renders.  Waits for them and clears the record. */
int ptg_last_kernel_busy(ptg_context* ctx, double busy_ms[8], double ms[8], uint32_t launches[8]);

/* Execution strategy of ptg_render*: 0 = wavefront pipeline (default:
 * camera / extend / shadow / shade kernels over compacted path queues),
 * 1 = megakernel (one work-item runs a whole path).  Both produce identical
 * bits. */
int ptg_set_pipeline(ptg_context* ctx, int pipeline);

/* Concurrency of the wavefront pipeline: 0 = every kernel on the context's
 * stream; 1 = the sky and shadow kernels on a second stream beside the walks;
 * 2 (default) = in addition two sample chunks in flight on their own stream
 * pairs, folded in sample order.  All levels produce identical bits. */
int ptg_set_concurrency(ptg_context* ctx, int level);

/* Device memory the wavefront path state may take: at most `percent` (5-70,
 * default 35) of the GPU's HBM per chunk pipeline, and never more than 85% of
 * what is free.  A smaller share means smaller sample chunks (more launches);
 * the bits do not change. */
int ptg_set_hbm_share(ptg_context* ctx, int percent);

/* Live paths per sample chunk and pipeline: at most 2^log2_paths (16-28,
 * default 27: 2^27 x 380 B = ~51 GB of path state per pipeline).  A renderer
 * that owns the GPU takes 28 with a 40% HBM share (4 chunks of 256 spp at
 * 1280x720x1024, ~71% of HBM); the bits do not change. */
int ptg_set_chunk_paths(ptg_context* ctx, int log2_paths);

/* Environment knobs read once by ptg_context_create (timing experiments;
 * no result bit depends on any of them; a malformed or out-of-range value is
 * ignored).  An embedding application that must not have its memory use or
 * launch shape changed from outside should leave them unset:
 *   PTG_CHUNK_LOG2              initial ptg_set_chunk_paths value (16-28)
 *   PTG_HBM_SHARE               initial ptg_set_hbm_share value (5-70)
 *   PTG_WALK_RESIDENT[_ANY]     closest-hit [any-hit] walk blocks resident per
 *                               CU (pads the blocks' LDS; 0-64)
 *   PTG_WALK_BLOCKS[_ANY]       closest-hit [any-hit] walk blocks launched per
 *                               CU (0-64)
 * The ptg_set_* calls after ptg_context_create override the first two. */

/* Synchronise the context's stream. */
int ptg_synchronize(ptg_context* ctx);

/* Device memory helpers for C callers without a device allocator. */
int ptg_device_alloc(ptg_context* ctx, size_t bytes, void** out);
int ptg_device_free(ptg_context* ctx, void* p);
int ptg_memcpy_d2h(ptg_context* ctx, void* dst, const void* src, size_t bytes);

#ifdef __cplusplus
}
#endif
#endif /* PTG_H */
