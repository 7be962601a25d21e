// SLP root-cause probe, part 2: the walk's triangle test
// alone.  tri_accept (device/path_tracer.h) on seeded rays and triangles, in
// the two forms the walker instantiates it - the closest-hit form (u, v, t,
// back and the verdict) and the any-hit form (the verdict only) - compiled
// once with the SLP vectoriser and once without (tools/slp_tri.sh); the two
// binaries' outputs must be the same bytes.
// Usage: slp_tri <out.bin> [n]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>
#include <random>
#include <vector>
#include "device/path_tracer.h"

using namespace ptg::dm;

struct Case {
    float org[3], d[3], p[9], tmin, tmax;
};

// the walker's per-BLAS setup (BlockWalker::enter): axis and S from the ray
__device__ __forceinline__ void setup(const Case& c, f3& org, int& axis, f3& S)
{
    org = V3(c.org[0], c.org[1], c.org[2]);
    const f3 d = V3(c.d[0], c.d[1], c.d[2]);
    tri_preprocess(d, axis, S);
}

__global__ void k_full(uint32_t n, const Case* __restrict__ cs, uint32_t* __restrict__ out)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if(i >= n) return;
    const Case c = cs[i];
    f3 org, S;
    int axis;
    setup(c, org, axis, S);
    float u = 0, v = 0, t = 0;
    bool back = false;
    const bool ok = tri_accept(org, axis, S, V3(c.p[0], c.p[1], c.p[2]), V3(c.p[3], c.p[4], c.p[5]),
                               V3(c.p[6], c.p[7], c.p[8]), c.tmin, c.tmax, u, v, t, back);
    uint32_t* w = out + size_t(i) * 5;
    w[0] = ok;
    w[1] = ok ? __float_as_uint(u) : 0u;
    w[2] = ok ? __float_as_uint(v) : 0u;
    w[3] = ok ? __float_as_uint(t) : 0u;
    w[4] = ok ? back : 0u;
}

__global__ void k_any(uint32_t n, const Case* __restrict__ cs, uint32_t* __restrict__ out)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if(i >= n) return;
    const Case c = cs[i];
    f3 org, S;
    int axis;
    setup(c, org, axis, S);
    float u, v, t;
    bool back;
    out[i] = tri_accept(org, axis, S, V3(c.p[0], c.p[1], c.p[2]), V3(c.p[3], c.p[4], c.p[5]),
                        V3(c.p[6], c.p[7], c.p[8]), c.tmin, c.tmax, u, v, t, back);
}

int main(int argc, char** argv)
{
    if(argc < 2) { fprintf(stderr, "usage: slp_tri out.bin [n]\n"); return 2; }
    const uint32_t n = argc > 2 ? uint32_t(atoi(argv[2])) : (1u << 22);
    std::vector<Case> cs(n);
    std::mt19937 g(450);
    std::uniform_real_distribution<float> U(-1.0f, 1.0f), P(0.0f, 1.0f);
    for(Case& c: cs)
    {   // a ray from near the origin towards a triangle around a point at distance 1..100
        const float dist = 1.0f + 99.0f * P(g);
        float dir[3] = {U(g), U(g), U(g)};
        const float len = std::sqrt(dir[0] * dir[0] + dir[1] * dir[1] + dir[2] * dir[2]) + 1e-6f;
        const float size = 0.05f + 2.0f * P(g);
        for(int k = 0; k < 3; ++k)
        {
            c.org[k] = 0.1f * U(g);
            c.d[k] = dir[k] / len;
            const float centre = c.org[k] + c.d[k] * dist + 0.5f * size * U(g);
            for(int j = 0; j < 3; ++j) c.p[j * 3 + k] = centre + size * U(g);
        }
        c.tmin = 0.0f;
        c.tmax = P(g) < 0.5f ? 1e30f : dist * (0.5f + P(g));
    }
    Case* dc = nullptr;
    uint32_t* dout = nullptr;
    if(hipMalloc(&dc, n * sizeof(Case)) != hipSuccess || hipMalloc(&dout, size_t(n) * 6 * 4) != hipSuccess) return 2;
    if(hipMemcpy(dc, cs.data(), n * sizeof(Case), hipMemcpyHostToDevice) != hipSuccess) return 2;
    const uint32_t grid = (n + 255) / 256;
    hipLaunchKernelGGL(k_full, dim3(grid), dim3(256), 0, nullptr, n, dc, dout);
    hipLaunchKernelGGL(k_any, dim3(grid), dim3(256), 0, nullptr, n, dc, dout + size_t(n) * 5);
    std::vector<uint32_t> out(size_t(n) * 6);
    if(hipMemcpy(out.data(), dout, out.size() * 4, hipMemcpyDeviceToHost) != hipSuccess) return 2;
    size_t accepted = 0, any = 0;
    for(uint32_t i = 0; i < n; ++i) accepted += out[size_t(i) * 5], any += out[size_t(n) * 5 + i];
    FILE* f = fopen(argv[1], "wb");
    if(!f || fwrite(out.data(), 4, out.size(), f) != out.size()) return 2;
    fclose(f);
    printf("%u cases: %zu accepted (closest-hit form), %zu (any-hit form)\n", n, accepted, any);
    return 0;
}
