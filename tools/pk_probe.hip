// Root-cause probe for the SLP divergence: do gfx950's
// packed-FP32 instructions, in the operand forms the SLP vectoriser emitted
// for the walk (ROCm 7.2, -O3), give the same bits
// per lane as the scalar IEEE operations they replace?  Each form is issued
// through inline asm on random and special inputs (normals, denormals,
// zeros, infinities, NaN) and compared with the scalar expression computed
// with v_fma_f32 / v_mul_f32 / v_add_f32.
//   fma_inl1   v_pk_fma_f32 D, A, B, 1.0 op_sel_hi:[1,1,0] neg_lo:[1,0,0] neg_hi:[1,0,0]
//              (rcp_nr's Newton residual fma(-x, r, 1))
//   fma        v_pk_fma_f32 D, A, B, C
//   mul_bcast  v_pk_mul_f32 D, A, B op_sel_hi:[1,0]           (A * B.lo)
//   mul_hi     v_pk_mul_f32 D, A, B op_sel:[0,1]              (A * B.hi)
//   sub_bcast  v_pk_add_f32 D, A, B op_sel_hi:[1,0] neg_lo:[0,1] neg_hi:[0,1]   (A - B.lo)
//   sub_swap   v_pk_add_f32 D, A, A op_sel:[0,1] op_sel_hi:[1,0] neg_lo:[0,1] neg_hi:[0,1]
//   mul_neg    v_pk_mul_f32 D, A, B op_sel_hi:[0,1] neg_lo:[0,1] neg_hi:[0,1]  (A.lo * -B)
//   add        v_pk_add_f32 D, A, B
// Usage (GPU box): hipcc --offload-arch=gfx950 -O2 -ffp-contract=off -fno-slp-vectorize tools/pk_probe.hip -o pk_probe
//                  && ./pk_probe   (no SLP: scalar() must stay scalar)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstring>
#include <vector>

typedef float v2f __attribute__((ext_vector_type(2)));

enum { F_FMA_INL1, F_FMA, F_MUL_BCAST, F_MUL_HI, F_SUB_BCAST, F_SUB_SWAP, F_MUL_NEG, F_ADD, F_COUNT };
static const char* kNames[F_COUNT] = {"fma_inl1", "fma", "mul_bcast", "mul_hi", "sub_bcast", "sub_swap", "mul_neg", "add"};

__device__ __noinline__ v2f packed(int f, v2f a, v2f b, v2f c)
{
    v2f d;
    switch(f)
    {
    case F_FMA_INL1: asm volatile("v_pk_fma_f32 %0, %1, %2, 1.0 op_sel_hi:[1,1,0] neg_lo:[1,0,0] neg_hi:[1,0,0]" : "=v"(d) : "v"(a), "v"(b)); break;
    case F_FMA: asm volatile("v_pk_fma_f32 %0, %1, %2, %3" : "=v"(d) : "v"(a), "v"(b), "v"(c)); break;
    case F_MUL_BCAST: asm volatile("v_pk_mul_f32 %0, %1, %2 op_sel_hi:[1,0]" : "=v"(d) : "v"(a), "v"(b)); break;
    case F_MUL_HI: asm volatile("v_pk_mul_f32 %0, %1, %2 op_sel:[0,1]" : "=v"(d) : "v"(a), "v"(b)); break;
    case F_SUB_BCAST: asm volatile("v_pk_add_f32 %0, %1, %2 op_sel_hi:[1,0] neg_lo:[0,1] neg_hi:[0,1]" : "=v"(d) : "v"(a), "v"(b)); break;
    case F_SUB_SWAP: asm volatile("v_pk_add_f32 %0, %1, %1 op_sel:[0,1] op_sel_hi:[1,0] neg_lo:[0,1] neg_hi:[0,1]" : "=v"(d) : "v"(a)); break;
    case F_MUL_NEG: asm volatile("v_pk_mul_f32 %0, %1, %2 op_sel_hi:[0,1] neg_lo:[0,1] neg_hi:[0,1]" : "=v"(d) : "v"(a), "v"(b)); break;
    default: asm volatile("v_pk_add_f32 %0, %1, %2" : "=v"(d) : "v"(a), "v"(b)); break;
    }
    return d;
}

// what each form must compute, per lane, with scalar IEEE operations
__device__ __noinline__ v2f scalar(int f, v2f a, v2f b, v2f c)
{
    switch(f)
    {
    case F_FMA_INL1: return v2f{__builtin_fmaf(-a.x, b.x, 1.0f), __builtin_fmaf(-a.y, b.y, 1.0f)};
    case F_FMA: return v2f{__builtin_fmaf(a.x, b.x, c.x), __builtin_fmaf(a.y, b.y, c.y)};
    case F_MUL_BCAST: return v2f{a.x * b.x, a.y * b.x};
    case F_MUL_HI: return v2f{a.x * b.y, a.y * b.y};
    case F_SUB_BCAST: return v2f{a.x - b.x, a.y - b.x};
    case F_SUB_SWAP: { const float lo = a.x - a.y, hi = a.y - a.x; return v2f{lo, hi}; }
    case F_MUL_NEG: return v2f{a.x * -b.x, a.x * -b.y};
    default: return v2f{a.x + b.x, a.y + b.y};
    }
}

__global__ void k_probe(int f, const v2f* a, const v2f* b, const v2f* c, uint32_t n, v2f* got, v2f* want)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if(i >= n) return;
    got[i] = packed(f, a[i], b[i], c[i]);
    want[i] = scalar(f, a[i], b[i], c[i]);
}

static uint32_t rng(uint64_t& s)
{
    s = s * 6364136223846793005ull + 1442695040888963407ull;
    return uint32_t(s >> 32);
}

static float pick(uint64_t& s)
{
    const uint32_t k = rng(s) % 16;
    uint32_t u = rng(s);
    if(k == 0) u &= 0x807FFFFFu;                 // denormal (or zero)
    else if(k == 1) u = (u & 0x80000000u) | 0x00800000u | (u & 0x7Fu);   // tiny normal
    else if(k == 2) u = (u & 0x80000000u) | 0x7F800000u;                 // infinity
    else if(k == 3) u = 0x7FC00000u;             // NaN
    else if(k < 9) u = (u & 0x807FFFFFu) | ((100u + (rng(s) % 56u)) << 23);   // moderate magnitudes
    float x;
    memcpy(&x, &u, 4);
    return x;
}

int main()
{
    const uint32_t n = 1u << 22;
    std::vector<v2f> a(n), b(n), c(n), got(n), want(n);
    uint64_t s = 12345;
    for(uint32_t i = 0; i < n; ++i)
    {
        a[i] = v2f{pick(s), pick(s)};
        b[i] = v2f{pick(s), pick(s)};
        c[i] = v2f{pick(s), pick(s)};
    }
    v2f *da, *db, *dc, *dg, *dw;
    const size_t bytes = size_t(n) * sizeof(v2f);
    if(hipMalloc(&da, bytes) || hipMalloc(&db, bytes) || hipMalloc(&dc, bytes) || hipMalloc(&dg, bytes) || hipMalloc(&dw, bytes))
        return 2;
    if(hipMemcpy(da, a.data(), bytes, hipMemcpyHostToDevice) || hipMemcpy(db, b.data(), bytes, hipMemcpyHostToDevice) ||
       hipMemcpy(dc, c.data(), bytes, hipMemcpyHostToDevice))
        return 2;
    int status = 0;
    for(int f = 0; f < F_COUNT; ++f)
    {
        hipLaunchKernelGGL(k_probe, dim3((n + 255) / 256), dim3(256), 0, nullptr, f, da, db, dc, n, dg, dw);
        if(hipMemcpy(got.data(), dg, bytes, hipMemcpyDeviceToHost) || hipMemcpy(want.data(), dw, bytes, hipMemcpyDeviceToHost))
            return 2;
        uint64_t mis[2] = {0, 0}, denorm_in = 0;
        int shown = 0;
        for(uint32_t i = 0; i < n; ++i)
            for(int h = 0; h < 2; ++h)
            {
                const float g = h ? got[i].y : got[i].x, w = h ? want[i].y : want[i].x;
                uint32_t gu, wu;
                memcpy(&gu, &g, 4);
                memcpy(&wu, &w, 4);
                if(gu == wu || (g != g && w != w)) continue;
                ++mis[h];
                if(shown++ < 6)
                    printf("  %s lane %s: a=(%a,%a) b=(%a,%a) c=(%a,%a): packed %a scalar %a\n", kNames[f], h ? "hi" : "lo",
                           a[i].x, a[i].y, b[i].x, b[i].y, c[i].x, c[i].y, g, w);
            }
        (void)denorm_in;
        printf("%-10s %u pairs: %llu lo-lane and %llu hi-lane mismatches\n", kNames[f], n, (unsigned long long)mis[0],
               (unsigned long long)mis[1]);
        if(mis[0] || mis[1]) status = 1;
    }
    return status;
}
