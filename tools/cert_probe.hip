// How often do the shading kernels' rounding certificates fail (ref_math.h,
// MathFast)?  Runs the atmosphere integrals, the Fresnel term and the GGX
// sample on seeded random inputs with a policy that counts, per certificate
// site, the evaluations and the failures, and records the first failing
// values; compares each certified float with the exact (MathExact) one where
// the certificate held (they must be equal).
// Usage: cert_probe [n]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include "device/path_tracer.h"

using namespace ptg::dm;

struct MathProbe {
    static constexpr bool kFast = true;
    uint32_t fail_mask = 0;
    unsigned long long* ctr;   // [site] evaluations, [CS_COUNT + site] failures
    double* ex;                // [site * 4 + k] first failing values
    __device__ void check(bool certain, double v, int site)
    {
        atomicAdd(ctr + site, 1ull);
        if(!certain)
        {
            fail_mask |= 1u << site;
            const unsigned long long k = atomicAdd(ctr + CS_COUNT + site, 1ull);
            if(k < 4) ex[site * 4 + k] = v;
        }
    }
};

__device__ uint32_t hash(uint32_t x)
{
    x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
    return x;
}
__device__ float unit(uint32_t& s) { s = hash(s + 0x9e3779b9u); return float(s >> 8) * (1.0f / 16777216.0f); }

__global__ void k_probe(uint32_t n, unsigned long long* ctr, double* ex, uint32_t* mismatch)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if(i >= n) return;
    uint32_t s = hash(i * 7919u + 1u);
    MathProbe mp{0, ctr, ex};
    MathExact mx;
    // the sky of a path: origin near the ground, a random direction, the sun
    const f3 pos = V3(200.0f * (unit(s) - 0.5f), 1.0f + 300.0f * unit(s), 200.0f * (unit(s) - 0.5f));
    const f3 view = normalize(V3(unit(s) - 0.5f, unit(s) - 0.3f, unit(s) - 0.5f));
    Light L;
    L.dir = normalize(V3(0.3f, 0.2f + unit(s), 0.1f));
    L.color = V3(1.0f, 1.0f, 1.0f);
    L.cos = 0.9999f;
    u4 seed{hash(s), hash(s + 1), hash(s + 2), hash(s + 3)};
    u4 seed2 = seed;
    const float tmax = unit(s) < 0.5f ? -1.0f : 1e4f * unit(s);
    f3 a0, i0, a1, i1;
    mp.fail_mask = 0;
    atmosphere_scattering(seed, L, pos, view, tmax, a0, i0, mp);
    const bool f_scatter = mp.fail_mask != 0;
    atmosphere_scattering(seed2, L, pos, view, tmax, a1, i1, mx);
    if(!f_scatter && (a0.x != a1.x || a0.y != a1.y || a0.z != a1.z || i0.x != i1.x || i0.y != i1.y || i0.z != i1.z))
        atomicAdd(mismatch, 1u);
    mp.fail_mask = 0;
    const f3 t0 = atmosphere_attenuation(unit(s), pos, view, MAX_RAY_DIST, mp);
    const bool f_att = mp.fail_mask != 0;
    const f3 t1 = atmosphere_attenuation(0.0f, pos, view, MAX_RAY_DIST, mx);
    (void)f_att; (void)t0; (void)t1;
    // a material: Fresnel, the GGX sample
    const float vdh = 2.0f * unit(s) - 1.0f, f0 = 0.04f * unit(s), rough = unit(s);
    mp.fail_mask = 0;
    const float fr0 = fresnel_att(vdh, f0, 1.0f + unit(s), rough, mp);
    const float fr1 = fresnel_att(vdh, f0, 1.0f + 0.0f, rough, mx);
    (void)fr0; (void)fr1;
    const f3 gv = ggx_vndf(view, rough, f2{unit(s), unit(s)}, mp);
    (void)gv;
    // path-space regularisation (bounce_tail): bpdf log-uniform in [1e-4, 1e4], r in (0, 1]
    const float bpdf = powf(10.0f, 8.0f * unit(s) - 4.0f);
    const float rr = unit(s) < 0.3f ? 1.0f : unit(s);
    const float g0 = times_one_minus_div_pow(rr, (double)REGULARIZATION_GAMMA, (double)bpdf, 0.25, mp);
    const float g1 = times_one_minus_div_pow(rr, (double)REGULARIZATION_GAMMA, (double)bpdf, 0.25, mx);
    if(!(mp.fail_mask & (1u << CS_TIMES_ONE_MINUS_DIV_POW)) && g0 != g1) atomicAdd(mismatch, 1u);
}

int main(int argc, char** argv)
{
    const uint32_t n = argc > 1 ? uint32_t(atoi(argv[1])) : (1u << 20);
    unsigned long long* ctr;
    double* ex;
    uint32_t* mism;
    if(hipMalloc(&ctr, 2 * CS_COUNT * 8) != hipSuccess || hipMalloc(&ex, CS_COUNT * 4 * 8) != hipSuccess ||
       hipMalloc(&mism, 4) != hipSuccess)
        return 2;
    hipMemset(ctr, 0, 2 * CS_COUNT * 8);
    hipMemset(ex, 0, CS_COUNT * 4 * 8);
    hipMemset(mism, 0, 4);
    hipLaunchKernelGGL(k_probe, dim3((n + 255) / 256), dim3(256), 0, nullptr, n, ctr, ex, mism);
    unsigned long long h[2 * CS_COUNT];
    double hx[CS_COUNT * 4];
    uint32_t hm = 0;
    if(hipMemcpy(h, ctr, sizeof(h), hipMemcpyDeviceToHost) != hipSuccess || hipMemcpy(hx, ex, sizeof(hx), hipMemcpyDeviceToHost) ||
       hipMemcpy(&hm, mism, 4, hipMemcpyDeviceToHost))
        return 2;
    static const char* names[CS_COUNT] = {"acc_exp", "exp_times", "add_mul_pow", "div_mul_pow", "times_cos", "times_sin",
                                          "times_one_minus_div_pow"};
    for(int k = 0; k < CS_COUNT; ++k)
    {
        printf("%-26s evaluations %12llu failures %10llu (%.3g)", names[k], h[k], h[CS_COUNT + k],
               h[k] ? double(h[CS_COUNT + k]) / double(h[k]) : 0.0);
        for(int j = 0; j < 4 && j < (int)h[CS_COUNT + k]; ++j)
        {
            uint64_t u;
            memcpy(&u, &hx[k * 4 + j], 8);
            printf("  %.9g (0x%016llx)", hx[k * 4 + j], (unsigned long long)u);
        }
        printf("\n");
    }
    printf("certified scattering results differing from the exact ones: %u of %u\n", hm, n);
    return hm ? 1 : 0;
}
