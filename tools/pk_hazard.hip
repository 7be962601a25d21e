// Root-cause probe for the SLP divergence, part 2 (see tools/pk_probe.hip,
// DESIGN.md section 8): the instruction sequence ROCm 7.2 emitted for the
// triangle test's cross product in the any-hit walk of k_rays (-O3 with SLP,
// -g build; ref_math.h:44 cross() inlined into tri_accept, path_tracer.h:76-83),
// replayed verbatim with its own registers - no wait states beyond the
// compiler's - and again with an s_nop after every instruction.  Each result
// is compared with the same arithmetic done by scalar VALU instructions.
//
//   v_mov_b32    v32, v16
//   v_pk_mov_b32 v[0:1], v[28:29], v[26:27] op_sel:[1,0]
//   v_mov_b32    v33, v23
//   v_pk_mul_f32 v[0:1], v[0:1], v[32:33]
//   v_pk_mul_f32 v[22:23], v[26:27], v[22:23]
//   v_pk_mul_f32 v[16:17], v[28:29], v[16:17] neg_lo:[0,1] neg_hi:[0,1]
//   v_pk_add_f32 v[0:1], v[0:1], v[0:1] op_sel:[0,1] op_sel_hi:[1,0] neg_lo:[0,1] neg_hi:[0,1]
//   v_pk_add_f32 v[16:17], v[22:23], v[16:17]
//   s_nop 0
//   v_add_f32    v1, v17, v0
//   v_add_f32    v5, v16, v1
//
// Usage (GPU box): hipcc --offload-arch=gfx950 -O2 -ffp-contract=off -fno-slp-vectorize tools/pk_hazard.hip -o pk_hazard && ./pk_hazard
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstring>
#include <vector>

struct In { float v16, v17, v22, v23, v26, v27, v28, v29; };
struct Out { float v0, v1, v5, v16, v17; };

#define LOADS                                                                                        \
    "v_mov_b32 v16, %5\n v_mov_b32 v17, %6\n v_mov_b32 v22, %7\n v_mov_b32 v23, %8\n"                \
    "v_mov_b32 v26, %9\n v_mov_b32 v27, %10\n v_mov_b32 v28, %11\n v_mov_b32 v29, %12\n s_nop 4\n"
#define STORES "s_nop 4\n v_mov_b32 %0, v0\n v_mov_b32 %1, v1\n v_mov_b32 %2, v5\n v_mov_b32 %3, v16\n v_mov_b32 %4, v17\n"
#define CLOBBERS "v0", "v1", "v5", "v16", "v17", "v22", "v23", "v26", "v27", "v28", "v29", "v32", "v33"

__global__ void k_seq(int variant, const In* __restrict__ in, Out* __restrict__ out, uint32_t n)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if(i >= n) return;
    const In a = in[i];
    Out o;
    if(variant == 0)
        asm volatile(LOADS
                     "v_mov_b32 v32, v16\n"
                     "v_pk_mov_b32 v[0:1], v[28:29], v[26:27] op_sel:[1,0]\n"
                     "v_mov_b32 v33, v23\n"
                     "v_pk_mul_f32 v[0:1], v[0:1], v[32:33]\n"
                     "v_pk_mul_f32 v[22:23], v[26:27], v[22:23]\n"
                     "v_pk_mul_f32 v[16:17], v[28:29], v[16:17] neg_lo:[0,1] neg_hi:[0,1]\n"
                     "v_pk_add_f32 v[0:1], v[0:1], v[0:1] op_sel:[0,1] op_sel_hi:[1,0] neg_lo:[0,1] neg_hi:[0,1]\n"
                     "v_pk_add_f32 v[16:17], v[22:23], v[16:17]\n"
                     "s_nop 0\n"
                     "v_add_f32 v1, v17, v0\n"
                     "v_add_f32 v5, v16, v1\n" STORES
                     : "=v"(o.v0), "=v"(o.v1), "=v"(o.v5), "=v"(o.v16), "=v"(o.v17)
                     : "v"(a.v16), "v"(a.v17), "v"(a.v22), "v"(a.v23), "v"(a.v26), "v"(a.v27), "v"(a.v28), "v"(a.v29)
                     : CLOBBERS);
    else
        asm volatile(LOADS
                     "v_mov_b32 v32, v16\n s_nop 4\n"
                     "v_pk_mov_b32 v[0:1], v[28:29], v[26:27] op_sel:[1,0]\n s_nop 4\n"
                     "v_mov_b32 v33, v23\n s_nop 4\n"
                     "v_pk_mul_f32 v[0:1], v[0:1], v[32:33]\n s_nop 4\n"
                     "v_pk_mul_f32 v[22:23], v[26:27], v[22:23]\n s_nop 4\n"
                     "v_pk_mul_f32 v[16:17], v[28:29], v[16:17] neg_lo:[0,1] neg_hi:[0,1]\n s_nop 4\n"
                     "v_pk_add_f32 v[0:1], v[0:1], v[0:1] op_sel:[0,1] op_sel_hi:[1,0] neg_lo:[0,1] neg_hi:[0,1]\n s_nop 4\n"
                     "v_pk_add_f32 v[16:17], v[22:23], v[16:17]\n s_nop 4\n"
                     "v_add_f32 v1, v17, v0\n s_nop 4\n"
                     "v_add_f32 v5, v16, v1\n" STORES
                     : "=v"(o.v0), "=v"(o.v1), "=v"(o.v5), "=v"(o.v16), "=v"(o.v17)
                     : "v"(a.v16), "v"(a.v17), "v"(a.v22), "v"(a.v23), "v"(a.v26), "v"(a.v27), "v"(a.v28), "v"(a.v29)
                     : CLOBBERS);
    out[i] = o;
}

// the same arithmetic, one IEEE operation at a time
static Out expected(const In& a)
{
    const float p0 = a.v29 * a.v16, p1 = a.v26 * a.v23;          // v[0:1] = (v29, v26) * (v16, v23)
    const float q22 = a.v26 * a.v22, q23 = a.v27 * a.v23;        // v[22:23] = v[26:27] * v[22:23]
    const float r16 = a.v28 * -a.v16, r17 = a.v29 * -a.v17;      // v[16:17] = v[28:29] * -v[16:17]
    const float s0 = p0 - p1, s1 = p1 - p0;                      // v[0:1] = (v0 - v1, v1 - v0)
    const float t16 = q22 + r16, t17 = q23 + r17;
    const float u1 = t17 + s0;
    const float u5 = t16 + u1;
    return Out{s0, u1, u5, t16, t17};
}

static float rnd(uint64_t& s)
{
    s = s * 6364136223846793005ull + 1442695040888963407ull;
    const uint32_t u = uint32_t(s >> 32);
    return (float)((int32_t)(u % 2000001u) - 1000000) / 1000.0f;
}

int main()
{
    const uint32_t n = 1u << 20;
    std::vector<In> in(n);
    uint64_t s = 7;
    for(auto& a: in) a = In{rnd(s), rnd(s), rnd(s), rnd(s), rnd(s), rnd(s), rnd(s), rnd(s)};
    In* din;
    Out* dout;
    if(hipMalloc(&din, n * sizeof(In)) || hipMalloc(&dout, n * sizeof(Out))) return 2;
    if(hipMemcpy(din, in.data(), n * sizeof(In), hipMemcpyHostToDevice)) return 2;
    std::vector<Out> out(n);
    const char* names[2] = {"compiler's sequence", "s_nop 4 after every instruction"};
    int status = 0;
    for(int v = 0; v < 2; ++v)
    {
        hipLaunchKernelGGL(k_seq, dim3(n / 256), dim3(256), 0, nullptr, v, din, dout, n);
        if(hipMemcpy(out.data(), dout, n * sizeof(Out), hipMemcpyDeviceToHost)) return 2;
        uint64_t bad[5] = {0, 0, 0, 0, 0};
        int shown = 0;
        for(uint32_t i = 0; i < n; ++i)
        {
            const Out e = expected(in[i]);
            const float* g = &out[i].v0;
            const float* w = &e.v0;
            bool any = false;
            for(int k = 0; k < 5; ++k)
                if(memcmp(&g[k], &w[k], 4) != 0) { ++bad[k]; any = true; }
            if(any && shown++ < 4)
                printf("  %s: in v16..v29 = %g %g %g %g %g %g %g %g -> v0 %g/%g v1 %g/%g v5 %g/%g v16 %g/%g v17 %g/%g\n",
                       names[v], in[i].v16, in[i].v17, in[i].v22, in[i].v23, in[i].v26, in[i].v27, in[i].v28, in[i].v29,
                       g[0], w[0], g[1], w[1], g[2], w[2], g[3], w[3], g[4], w[4]);
        }
        printf("%-34s mismatches: v0 %llu v1 %llu v5 %llu v16 %llu v17 %llu of %u\n", names[v],
               (unsigned long long)bad[0], (unsigned long long)bad[1], (unsigned long long)bad[2],
               (unsigned long long)bad[3], (unsigned long long)bad[4], n);
        if(bad[0] | bad[1] | bad[2] | bad[3] | bad[4]) status = 1;
    }
    return status;
}
