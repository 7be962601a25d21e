// Second translation unit of the two-TU user library (tests/device_dropin/
// Makefile): a user library whose .hip files each include ptg_device.h must
// link - every definition the header makes is inline or has internal linkage.
#include "ptg_device.h"

namespace {
__global__ void k_user_tonemap2(uint32_t n, const ptg_float4* in, ptg_uchar4* out)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if(i >= n) return;
    ptg_float3 c;
    c.x = in[i].x;
    c.y = in[i].y;
    c.z = in[i].z;
    out[i] = tonemap_pixel(c);
}
} // namespace

extern "C" {
int user_selftest_tu2() { return ptg_device_selftest(); }

int user_tonemap_device_tu2(uint32_t n, const ptg_float4* in, ptg_uchar4* out)
{
    hipLaunchKernelGGL(k_user_tonemap2, dim3((n + 255) / 256), dim3(256), 0, nullptr, n, in, out);
    return hipDeviceSynchronize() == hipSuccess ? 0 : -1;
}
}
