/* pt_oracle.h - CPU restatement of the reference hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  This is the checker the GPU path is compared
 * against; only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
 * leg may load it.  The product (libptg.so) never links or calls it.
 *
 * Reference: Kalache-abdesattar/Path-Tracing...but-on-the-LUMI-cluster @ v1,
 * path_tracer.hh, ray_query.hh, math.hh (file:line cited per function in
 * pt_oracle.c).  Arrays are in the reference byte layout (see include/ptg.h).
 */
#ifndef PT_ORACLE_H
#define PT_ORACLE_H
#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
    const void* subframes;      /* subframe[]        (scene.hh:26-34, 160 B) */
    const void* instances;      /* tlas_instance[]   (bvh.hh:73-79, 160 B) */
    const void* nodes;          /* bvh_node[]        (24 B) */
    const void* links;          /* bvh_link[]        (8 B) */
    const uint32_t* indices;
    const void* pos;            /* float3[] (16 B) */
    const void* normal;         /* float3[] (16 B) */
    const void* albedo;         /* float4[] */
    const void* material;       /* float4[] */
} orc_scene;

typedef struct {
    uint32_t width, height, samples_per_pixel, max_bounces, student_id, samples_per_motion_blur_step;
} orc_config;

/* counters[0..7]: samples, node visits, triangle tests, BLAS entries, ray queries, closest-hit shades */
void orc_path_trace_pixel(const orc_scene* s, const orc_config* c, uint32_t x, uint32_t y, int32_t sample_index,
                          float out[4], uint64_t* counters);
void orc_tonemap_pixel(const float color[3], uint8_t out_bgra[4]);
void orc_pcg4d(uint32_t seed[4]);
void orc_uniform4(uint32_t seed[4], float out[4]);
/* ray = {o.xyz, d.xyz, tmin, tmax}; out = {bary.xyz, thit, instance, primitive, back_face, shadowed} */
void orc_trace_ray(const orc_scene* s, uint32_t subframe, const float ray[8], uint32_t out[8]);
/* baseline_render (main.cc:12-46) over a rectangle and sample range;
 * accum: [h][w][4] averaged radiance (divided by samples_per_pixel), bgra: [h][w][4] */
void orc_render_rect(const orc_scene* s, const orc_config* c, uint32_t x0, uint32_t y0, uint32_t w, uint32_t h,
                     uint32_t j0, uint32_t j1, float* accum, uint8_t* bgra, uint64_t* counters);

#ifdef __cplusplus
}
#endif
#endif
