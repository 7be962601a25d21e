// Exhaustive check of the device reciprocal used by the BVH walk
// (ref_math.h rcp_rn) against IEEE single-precision division 1.0f / x:
// every one of the 2^32 bit patterns, bit for bit.  The check runs once on
// the GPU box (tools/rcp_exhaustive.sh); it is what licenses rcp_rn in place
// of the division in a bit-exact hot path.
//
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -fno-fast-math
//         -fhip-fp32-correctly-rounded-divide-sqrt -I<pkg>/csrc tools/rcp_exhaustive.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstring>
#include "device/ref_math.h"

using ptg::dm::rcp_rn;

__global__ void k_check(uint64_t begin, uint64_t count, unsigned long long* mismatches, uint32_t* first)
{
    for(uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < count; i += (uint64_t)gridDim.x * blockDim.x)
    {
        const uint32_t u = uint32_t(begin + i);
        const float x = __uint_as_float(u);
        const float want = 1.0f / x;
        const float got = rcp_rn(x);
        const bool same = __float_as_uint(want) == __float_as_uint(got) || (want != want && got != got);
        if(!same)
        {
            const unsigned long long k = atomicAdd(mismatches, 1ull);
            if(k < 64) first[k] = u;
        }
    }
}

int main()
{
    unsigned long long* d_mis;
    uint32_t* d_first;
    if(hipMalloc(&d_mis, sizeof(unsigned long long)) != hipSuccess || hipMalloc(&d_first, 64 * 4) != hipSuccess)
    {
        printf("hipMalloc failed\n");
        return 2;
    }
    if(hipMemset(d_mis, 0, sizeof(unsigned long long)) != hipSuccess || hipMemset(d_first, 0, 64 * 4) != hipSuccess)
        return 2;
    const uint64_t total = 1ull << 32, slice = 1ull << 30;
    for(uint64_t b = 0; b < total; b += slice)
    {
        hipLaunchKernelGGL(k_check, dim3(4096), dim3(256), 0, nullptr, b, slice, d_mis, d_first);
        if(hipDeviceSynchronize() != hipSuccess)
        {
            printf("kernel failed\n");
            return 2;
        }
    }
    unsigned long long mis = 0;
    uint32_t first[64];
    if(hipMemcpy(&mis, d_mis, sizeof(mis), hipMemcpyDeviceToHost) != hipSuccess ||
       hipMemcpy(first, d_first, sizeof(first), hipMemcpyDeviceToHost) != hipSuccess)
        return 2;
    printf("rcp_rn vs 1.0f/x over all 2^32 inputs: %llu mismatches\n", mis);
    for(unsigned k = 0; k < mis && k < 64; ++k)
    {
        float x;
        std::memcpy(&x, &first[k], 4);
        printf("  0x%08x (%g)\n", first[k], x);
    }
    return mis == 0 ? 0 : 1;
}
