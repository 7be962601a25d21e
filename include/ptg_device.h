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
#include <string.h>
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

/* ---- ptg_device_selftest: known answers in the including translation unit -
 * The results above are the reference's bits only under the compile flags
 * named at the top of this header.  -ffast-math is refused at compile time;
 * the others leave no macro to test, so this self-test runs known-answer
 * checks compiled with the caller's own flags, on the caller's device, and
 * returns a bit mask of the checks that failed (0: all passed; negative: a
 * HIP error code, negated):
 *   bit 0  float a * b + c was contracted into an fma (-ffp-contract=off missing)
 *   bit 1  exp, bit 2 pow, bit 3 sin / cos: the device's glibc restatements
 *          against this host's libm on arguments where other libraries differ
 *   bit 4  tonemap_pixel on the device against the host's
 *   bit 5  fmin's tie rule (glibc: equal operands give the second)
 *   bit 6  float division and reciprocal, correctly rounded (the walk's
 *          reciprocals and -fhip-fp32-correctly-rounded-divide-sqrt)
 * The SLP vectoriser's divergence shows only inside a
 * whole BVH walk; tests/test_gpu_parity.py's ray records catch it. */
namespace ptg_selftest {
enum { kArgs = 8 };
struct Io {
    float a, b, c, fma_out;         /* contraction probe */
    float x[kArgs];                 /* library arguments */
    double exp_out[kArgs], pow_out[kArgs], sin_out[kArgs], cos_out[kArgs];
    ptg_float3 colors[kArgs];
    ptg_uchar4 tone_out[kArgs];
    float tie_out[2];
    float div_out[kArgs], rcp_out[kArgs];
};
/* internal linkage: several translation units of one library may include
 * this header (tests/device_dropin builds a two-TU library to check it) */
namespace {
__global__ void kernel(Io* io)
{
    if(threadIdx.x != 0 || blockIdx.x != 0) return;
    io->fma_out = io->a * io->b + io->c;
    for(int i = 0; i < kArgs; ++i)
    {
        const double d = (double)io->x[i];
        io->exp_out[i] = ptg::glibc::exp(d);
        io->pow_out[i] = ptg::glibc::pow(d, (double)(1.0f / 2.4f));
        io->sin_out[i] = ptg::glibc::sin(d);
        io->cos_out[i] = ptg::glibc::cos(d);
        io->tone_out[i] = tonemap_pixel(io->colors[i]);
        io->div_out[i] = io->a / io->x[i];
        io->rcp_out[i] = ptg::dm::rcp_rn(io->x[i]);
    }
    io->tie_out[0] = ptg::dm::gmin(io->c - io->c, -(io->c - io->c));   /* fmin(+0, -0): -0 */
    io->tie_out[1] = ptg::dm::gmax(-(io->c - io->c), io->c - io->c);   /* fmax(-0, +0): +0 */
}
} // namespace
inline bool same(double a, double b) { return memcmp(&a, &b, sizeof a) == 0; }
inline bool samef(float a, float b) { return memcmp(&a, &b, sizeof a) == 0; }
} // namespace ptg_selftest

static inline int ptg_device_selftest(hipStream_t stream = nullptr)
{
    using namespace ptg_selftest;
    Io h;
    memset(&h, 0, sizeof h);
    h.a = 1.0f + 0x1p-12f; h.b = 1.0f + 0x1p-12f; h.c = -(1.0f + 0x1p-11f);   /* fused: 2^-24, unfused: 0 */
    /* arguments where ocml's double differs from glibc's (profiles/r03_exhaustive) */
    const float xs[kArgs] = {0x1.58a68ap-24f, 0.00591448275f, 0.0040609352f, 1.7f, 3.0f, 0.7531f, 5.25f, 0x1.fffffep-1f};
    for(int i = 0; i < kArgs; ++i)
    {
        h.x[i] = xs[i];
        h.colors[i].x = xs[i] * 0.5f; h.colors[i].y = xs[i]; h.colors[i].z = xs[i] * 2.0f;
    }
    Io* d = nullptr;
    hipError_t e = hipMalloc(&d, sizeof(Io));
    if(e == hipSuccess) e = hipMemcpyAsync(d, &h, sizeof(Io), hipMemcpyHostToDevice, stream);
    if(e == hipSuccess)
    {
        hipLaunchKernelGGL(ptg_selftest::kernel, dim3(1), dim3(64), 0, stream, d);
        e = hipGetLastError();
    }
    Io r;
    if(e == hipSuccess) e = hipMemcpyAsync(&r, d, sizeof(Io), hipMemcpyDeviceToHost, stream);
    if(e == hipSuccess) e = hipStreamSynchronize(stream);
    if(d) (void)hipFree(d);
    if(e != hipSuccess) return -(int)e;
    int bad = 0;
    if(r.fma_out != 0.0f) bad |= 1;
    for(int i = 0; i < kArgs; ++i)
    {
        const double x = (double)h.x[i];
        if(!same(r.exp_out[i], exp(x))) bad |= 2;
        if(!same(r.pow_out[i], pow(x, (double)(1.0f / 2.4f)))) bad |= 4;
        if(!same(r.sin_out[i], sin(x)) || !same(r.cos_out[i], cos(x))) bad |= 8;
        const ptg_uchar4 t = tonemap_pixel(h.colors[i]);
        if(memcmp(&t, &r.tone_out[i], sizeof t) != 0) bad |= 16;
        if(!samef(r.div_out[i], h.a / h.x[i]) || !samef(r.rcp_out[i], 1.0f / h.x[i])) bad |= 64;
    }
    if(!samef(r.tie_out[0], -0.0f) || !samef(r.tie_out[1], 0.0f)) bad |= 32;
    return bad;
}

#endif /* PTG_DEVICE_H */
