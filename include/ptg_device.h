/* ptg_device.h - the reference's plugin functions with their own signatures,
 * for HIP code that keeps the reference's per-pixel loop on the GPU.
 *
 * The reference's plugin API is two C-callable inline functions
 * (README.md:38-39):
 *
 *   float3 path_trace_pixel(uint2 xy, int sample_index, const subframe*,
 *       const tlas_instance*, const bvh_node*, const bvh_link*, const uint*,
 *       const float3*, const float3*, const float4*, const float4*);
 *                                                     path_tracer.hh:637-654
 *   uchar4 tonemap_pixel(float3 color);               path_tracer.hh:753
 *
 * This header provides both, same names, same argument meaning, over the
 * same reference-layout arrays (bvh.hh, mesh.hh, scene.hh; see ptg.h for the
 * byte layouts - ptg_float3 is 16 bytes), now resident in device memory:
 *
 *   __device__          ptg_float3 path_trace_pixel(xy, sample_index, 9 arrays)
 *   __host__ __device__ ptg_uchar4 tonemap_pixel(ptg_float3)
 *
 * path_trace_pixel walks the arrays exactly as ray_query.hh does (no
 * repacking, device/path_tracer.h: RefScene) and returns the reference's
 * float32 result bit for bit (tests/test_gpu_device_dropin.py).  The
 * reference bakes IMAGE_WIDTH/HEIGHT, MAX_BOUNCES, STUDENT_ID and
 * SAMPLES_PER_MOTION_BLUR_STEP in as macros (config.hh); here they come from
 * the render configuration set once with ptg_device_set_config() (one
 * __constant__ copy per translation unit), or explicitly through the
 * ptg_path_trace_pixel_cfg() overload.
 *
 * The frame-level fast path is ptg_render() (ptg.h), the wavefront pipeline
 * over repacked records; this header is the drop-in for code that wants the
 * per-sample function itself (route B).
 *
 * Compile the including file with hipcc for gfx950 and with the flags that
 * make the arithmetic the reference's IEEE arithmetic:
 *   hipcc --offload-arch=gfx950 -ffp-contract=off -fno-fast-math \
 *         -fhip-fp32-correctly-rounded-divide-sqrt -fno-slp-vectorize \
 *         -I<repo>/include -I<repo>/<package>/csrc
 */
#ifndef PTG_DEVICE_H
#define PTG_DEVICE_H

#if defined(__FAST_MATH__)
#error "ptg_device.h: the reference's results need IEEE arithmetic - compile without -ffast-math (see the flags above)"
#endif

#include <hip/hip_runtime.h>
#include <math.h>
#include "ptg.h"
#include "device/path_tracer.h"

/* The render configuration path_trace_pixel reads (config.hh's macros). */
static __constant__ ptg_render_config ptg_device_render_config;

/* Host: set the configuration of this translation unit's path_trace_pixel. */
static inline hipError_t ptg_device_set_config(const ptg_render_config* cfg, hipStream_t stream = nullptr)
{
    return hipMemcpyToSymbolAsync(HIP_SYMBOL(ptg_device_render_config), cfg, sizeof(ptg_render_config), 0,
                                  hipMemcpyHostToDevice, stream);
}

/* path_trace_pixel (path_tracer.hh:637-741) with an explicit configuration. */
__device__ inline ptg_float3 ptg_path_trace_pixel_cfg(const ptg_render_config& cfg, ptg_uint2 xy, int sample_index,
                                                      const ptg_subframe* subframes,
                                                      const ptg_tlas_instance* instances,
                                                      const ptg_bvh_node* node_array,
                                                      const ptg_bvh_link* link_array, const uint32_t* mesh_indices,
                                                      const ptg_float3* mesh_pos, const ptg_float3* mesh_normal,
                                                      const ptg_float4* mesh_albedo,
                                                      const ptg_float4* mesh_material)
{
    ptg::dm::RefScene sc;
    sc.subframes = reinterpret_cast<const uint8_t*>(subframes);
    sc.instances = reinterpret_cast<const uint8_t*>(instances);
    sc.nodes = reinterpret_cast<const float*>(node_array);
    sc.links = reinterpret_cast<const uint2*>(link_array);
    sc.indices = mesh_indices;
    sc.pos = reinterpret_cast<const float*>(mesh_pos);
    sc.normal = reinterpret_cast<const float*>(mesh_normal);
    sc.albedo = reinterpret_cast<const float*>(mesh_albedo);
    sc.material = reinterpret_cast<const float*>(mesh_material);
    sc.polygon = nullptr;
    sc.width = cfg.width;
    sc.height = cfg.height;
    sc.max_bounces = cfg.max_bounces;
    sc.student_id = cfg.student_id;
    sc.blur_step = cfg.samples_per_motion_blur_step;
    ptg::dm::Counters cnt;
    const ptg::dm::f3 c = ptg::dm::path_trace_sample<false>(sc, xy.x, xy.y, (int32_t)sample_index, cnt);
    ptg_float3 out;
    out.x = c.x;
    out.y = c.y;
    out.z = c.z;
    return out;
}

/* path_trace_pixel (path_tracer.hh:637-654): the reference's signature. */
__device__ inline ptg_float3 path_trace_pixel(ptg_uint2 xy, int sample_index, const ptg_subframe* subframes,
                                              const ptg_tlas_instance* instances, const ptg_bvh_node* node_array,
                                              const ptg_bvh_link* link_array, const uint32_t* mesh_indices,
                                              const ptg_float3* mesh_pos, const ptg_float3* mesh_normal,
                                              const ptg_float4* mesh_albedo, const ptg_float4* mesh_material)
{
    return ptg_path_trace_pixel_cfg(ptg_device_render_config, xy, sample_index, subframes, instances, node_array,
                                    link_array, mesh_indices, mesh_pos, mesh_normal, mesh_albedo, mesh_material);
}

/* The C library's pow, as the reference calls it: glibc's own algorithm on
 * the device (device/glibc_math.h), glibc itself on the host. */
__host__ __device__ inline double ptg_libm_pow(double x, double y)
{
#if defined(__HIP_DEVICE_COMPILE__)
    return ptg::glibc::pow(x, y);
#else
    return pow(x, y);
#endif
}

/* tonemap_pixel (path_tracer.hh:753-771): ACES fit, sRGB curve in double as
 * the reference computes it, clamp with glibc's fmin/fmax tie rule, BGRA. */
__host__ __device__ inline float ptg_tonemap_channel(float c)
{
    c = (c * (2.51f * c + 0.03f)) / (c * (2.43f * c + 0.59f) + 0.14f);
    c = c < 0.0031308f ? c * 12.92f : (float)(ptg_libm_pow((double)c, (double)(1.0f / 2.4f)) * (double)1.055f - (double)0.055f);
    c = (c > 0.0f || 0.0f != 0.0f) ? c : 0.0f;                        /* fmax(c, 0): ties -> 0 */
    c = (c < 1.0f || 1.0f != 1.0f) ? c : 1.0f;                        /* fmin(c, 1) */
    return c;
}

__host__ __device__ inline ptg_uchar4 tonemap_pixel(ptg_float3 color)
{
    ptg_uchar4 o;
    o.x = (uint8_t)roundf(ptg_tonemap_channel(color.z) * 255.0f);
    o.y = (uint8_t)roundf(ptg_tonemap_channel(color.y) * 255.0f);
    o.z = (uint8_t)roundf(ptg_tonemap_channel(color.x) * 255.0f);
    o.w = 255;
    return o;
}

#endif /* PTG_DEVICE_H */
