// A user's kernel built against include/ptg_device.h only: the reference's
// per-sample loop body kept on the GPU, calling path_trace_pixel and
// tonemap_pixel with the reference's own signatures over reference-layout
// arrays in device memory (test infrastructure for
// tests/test_gpu_device_dropin.py; the product library is not linked).
#include "ptg_device.h"

__global__ void k_user_samples(uint32_t n, const ptg_uint2* __restrict__ xy, const int32_t* __restrict__ js,
                               const ptg_subframe* subframes, const ptg_tlas_instance* instances,
                               const ptg_bvh_node* nodes, const ptg_bvh_link* links, const uint32_t* indices,
                               const ptg_float3* pos, const ptg_float3* normal, const ptg_float4* albedo,
                               const ptg_float4* material, ptg_float4* out)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if(i >= n) return;
    const ptg_float3 c = path_trace_pixel(xy[i], js[i], subframes, instances, nodes, links, indices, pos, normal,
                                          albedo, material);
    out[i].x = c.x;
    out[i].y = c.y;
    out[i].z = c.z;
    out[i].w = 0.0f;
}

__global__ void k_user_tonemap(uint32_t n, const ptg_float4* __restrict__ in, ptg_uchar4* __restrict__ out)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if(i >= n) return;
    ptg_float3 c;
    c.x = in[i].x;
    c.y = in[i].y;
    c.z = in[i].z;
    out[i] = tonemap_pixel(c);
}

extern "C" {

// ptg_device_selftest() compiled with this library's flags (ptg_device.h)
int user_selftest() { return ptg_device_selftest(); }

// All array pointers are DEVICE pointers; synchronous.
int user_path_trace(const ptg_render_config* cfg, uint32_t n, const ptg_uint2* xy, const int32_t* js,
                    const ptg_subframe* subframes, const ptg_tlas_instance* instances, const ptg_bvh_node* nodes,
                    const ptg_bvh_link* links, const uint32_t* indices, const ptg_float3* pos,
                    const ptg_float3* normal, const ptg_float4* albedo, const ptg_float4* material, ptg_float4* out)
{
    if(hipError_t e = ptg_device_set_config(cfg)) return -1000 - int(e);
    hipLaunchKernelGGL(k_user_samples, dim3((n + 127) / 128), dim3(128), 0, 0, n, xy, js, subframes, instances, nodes,
                       links, indices, pos, normal, albedo, material, out);
    if(hipError_t e = hipGetLastError()) return -2000 - int(e);
    return hipDeviceSynchronize() == hipSuccess ? 0 : -3;
}

int user_tonemap_device(uint32_t n, const ptg_float4* in, ptg_uchar4* out)
{
    hipLaunchKernelGGL(k_user_tonemap, dim3((n + 255) / 256), dim3(256), 0, 0, n, in, out);
    if(hipError_t e = hipGetLastError()) return -2000 - int(e);
    return hipDeviceSynchronize() == hipSuccess ? 0 : -3;
}

// HOST pointers: tonemap_pixel called on the host.
void user_tonemap_host(uint32_t n, const ptg_float4* in, ptg_uchar4* out)
{
    for(uint32_t i = 0; i < n; ++i)
    {
        ptg_float3 c;
        c.x = in[i].x;
        c.y = in[i].y;
        c.z = in[i].z;
        out[i] = tonemap_pixel(c);
    }
}

}
