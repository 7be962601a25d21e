// Exhaustive checks of the exact fast paths in ref_math.h against the IEEE
// single-precision operation they replace, on every one of the 2^32 input bit
// patterns, bit for bit (any NaN matches any NaN):
//   rcp_rn(x)        vs 1.0f / x        (the walk's reciprocals)
//   div_by(x, c, rc) vs x / c           (c = the Rayleigh and Mie scale heights)
//   sqrt_rn(x)       vs sqrtf(x)        (fsqrt: lengths, sphere tests, sampling)
// Run once on the GPU box (tools/exhaustive.sh); it is what licenses these
// functions in place of the IEEE operations in a bit-exact hot path.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstring>
#include "device/ref_math.h"

using namespace ptg::dm;

enum { OP_RCP, OP_DIV, OP_SQRT };

__global__ void k_check(int op, uint64_t begin, uint64_t count, float c, float rc, unsigned long long* mismatches, uint32_t* first)
{
    for(uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < count; i += (uint64_t)gridDim.x * blockDim.x)
    {
        const uint32_t u = uint32_t(begin + i);
        const float x = __uint_as_float(u);
        float want, got;
        if(op == OP_RCP) { want = 1.0f / x; got = rcp_rn(x); }
        else if(op == OP_DIV) { want = x / c; got = div_by(x, c, rc); }
        else { want = __builtin_sqrtf(x); got = sqrt_rn(x); }
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
    struct Case { int op; float c; const char* name; } cases[] = {
        {OP_RCP, 0.0f, "rcp_rn(x) vs 1.0f / x"},
        {OP_DIV, 7994.0f, "div_by(x, 7994) vs x / 7994"},    // RAYLEIGH_SCALE_HEIGHT (path_tracer.h)
        {OP_DIV, 1200.0f, "div_by(x, 1200) vs x / 1200"},    // MIE_SCALE_HEIGHT
        {OP_SQRT, 0.0f, "sqrt_rn(x) vs sqrtf(x)"},
    };
    unsigned long long* d_mis;
    uint32_t* d_first;
    if(hipMalloc(&d_mis, sizeof(unsigned long long)) != hipSuccess || hipMalloc(&d_first, 64 * 4) != hipSuccess)
    {
        printf("hipMalloc failed\n");
        return 2;
    }
    int status = 0;
    for(const Case& k : cases)
    {
        const float rc = k.op == OP_DIV ? 1.0f / k.c : 0.0f;
        if(hipMemset(d_mis, 0, sizeof(unsigned long long)) != hipSuccess || hipMemset(d_first, 0, 64 * 4) != hipSuccess)
            return 2;
        const uint64_t total = 1ull << 32, slice = 1ull << 30;
        for(uint64_t b = 0; b < total; b += slice)
        {
            hipLaunchKernelGGL(k_check, dim3(4096), dim3(256), 0, nullptr, k.op, b, slice, k.c, rc, d_mis, d_first);
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
        printf("%s over all 2^32 inputs: %llu mismatches\n", k.name, mis);
        for(unsigned j = 0; j < mis && j < 16; ++j)
        {
            float x;
            std::memcpy(&x, &first[j], 4);
            printf("  0x%08x (%g)\n", first[j], x);
        }
        if(mis) status = 1;
    }
    return status;
}
