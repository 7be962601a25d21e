// Exhaustive check of the constant-divisor division used by the atmosphere
// (ref_math.h div_by) against IEEE single-precision division x / c: every one
// of the 2^32 bit patterns of x, bit for bit, for each scale height the sky
// divides by.  Run once on the GPU box (tools/div_exhaustive.sh); it is what
// licenses div_by in place of the division in a bit-exact hot path.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstring>
#include "device/ref_math.h"

using ptg::dm::div_by;

__global__ void k_check(uint64_t begin, uint64_t count, float c, float rc, unsigned long long* mismatches, uint32_t* first)
{
    for(uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < count; i += (uint64_t)gridDim.x * blockDim.x)
    {
        const uint32_t u = uint32_t(begin + i);
        const float x = __uint_as_float(u);
        const float want = x / c;
        const float got = div_by(x, c, rc);
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
    const float divisors[] = {7994.0f, 1200.0f};   // RAYLEIGH_SCALE_HEIGHT, MIE_SCALE_HEIGHT (path_tracer.h)
    unsigned long long* d_mis;
    uint32_t* d_first;
    if(hipMalloc(&d_mis, sizeof(unsigned long long)) != hipSuccess || hipMalloc(&d_first, 64 * 4) != hipSuccess)
    {
        printf("hipMalloc failed\n");
        return 2;
    }
    int status = 0;
    for(float c : divisors)
    {
        const float rc = 1.0f / c;
        if(hipMemset(d_mis, 0, sizeof(unsigned long long)) != hipSuccess || hipMemset(d_first, 0, 64 * 4) != hipSuccess)
            return 2;
        const uint64_t total = 1ull << 32, slice = 1ull << 30;
        for(uint64_t b = 0; b < total; b += slice)
        {
            hipLaunchKernelGGL(k_check, dim3(4096), dim3(256), 0, nullptr, b, slice, c, rc, d_mis, d_first);
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
        printf("div_by(x, %g) vs x / %g over all 2^32 inputs: %llu mismatches\n", c, c, mis);
        for(unsigned k = 0; k < mis && k < 64; ++k)
        {
            float x;
            std::memcpy(&x, &first[k], 4);
            printf("  0x%08x (%g)\n", first[k], x);
        }
        if(mis) status = 1;
    }
    return status;
}
