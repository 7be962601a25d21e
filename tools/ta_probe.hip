// Vector-memory cost probe (gfx950): how long does one wave-level gather
// instruction occupy a CU's vector memory path, as a function of
//   * the number of active lanes (EXEC) of the instruction,
//   * the bytes per lane (dword / dwordx2 / dwordx4),
//   * how many distinct cache lines the lanes touch,
//   * where the lines are served from (table size: L2, Infinity Cache, HBM)?
// The BVH walk (k_wf_walk) issues divergent 16-byte gathers and runs with
// TA_BUSY at ~80% of its cycles; these numbers are the ceilings its roofline
// is drawn against (bench.py "roofline").
//
// Each thread issues ITERS independent loads from the table at hashed
// addresses; lanes >= active skip the load (EXEC-masked).  32 waves per CU.
// Prints ns per wave-instruction per CU.
//
// usage: ta_probe                       full sweep (64 MiB table)
//        ta_probe sizes                 random 64-B lines, 64 active lanes, dwordx4, by table size
//        ta_probe <MiB> <active> <mode> <bytes>   one configuration (for rocprofv3 --pmc passes)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>
#include <cstring>

constexpr int ITERS = 2048;

__device__ __forceinline__ uint32_t hash(uint32_t x)
{
    x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
    return x;
}

// mode 0: random 64 B line per lane; 1: lanes in groups of 4 share a 64 B line
// (consecutive 16 B); 2: every lane of the wave reads the same address
template<int BYTES>
__global__ __launch_bounds__(256) void k_probe(const uint8_t* __restrict__ table, uint32_t lines, int active, int mode,
                                               uint32_t salt, float* __restrict__ sink)
{
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    float acc = 0.0f;
    if((int)lane < active)
    {
        for(int i = 0; i < ITERS; ++i)
        {
            uint32_t key = mode == 2 ? wave * 131u + i : (mode == 1 ? (wave * 64u + (lane >> 2)) : (wave * 64u + lane));
            uint32_t line = hash(key * 2654435761u + i * 40503u + salt) % lines;
            uint32_t off = line * 64u + (mode == 1 ? (lane & 3u) * 16u : 0u);
            if(BYTES == 16)
            {
                const float4 v = *reinterpret_cast<const float4*>(table + off);
                acc += v.x + v.w;
            }
            else if(BYTES == 8)
            {
                const float2 v = *reinterpret_cast<const float2*>(table + off);
                acc += v.x + v.y;
            }
            else
                acc += *reinterpret_cast<const float*>(table + off);
        }
    }
    if(acc == 12345.678f) sink[0] = acc;   // keeps the loads
}

struct Probe {
    uint8_t* table = nullptr;
    float* sink = nullptr;
    int cus = 0;
};

template<int BYTES>
float run(const Probe& p, size_t table_bytes, int active, int mode)
{
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    const dim3 grid(p.cus * 8), block(256);
    const uint32_t lines = uint32_t(table_bytes / 64);
    hipLaunchKernelGGL(k_probe<BYTES>, grid, block, 0, 0, p.table, lines, active, mode, 1u, p.sink);   // warm
    (void)hipEventRecord(a);
    hipLaunchKernelGGL(k_probe<BYTES>, grid, block, 0, 0, p.table, lines, active, mode, 7u, p.sink);
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, a, b);
    (void)hipEventDestroy(a);
    (void)hipEventDestroy(b);
    const double instr_per_cu = 32.0 * ITERS;   // 32 waves per CU, ITERS loads each
    return float(ms * 1e6 / instr_per_cu);      // ns per wave-instruction per CU
}

float run_bytes(const Probe& p, size_t table_bytes, int active, int mode, int bytes)
{
    return bytes == 4 ? run<4>(p, table_bytes, active, mode)
                      : bytes == 8 ? run<8>(p, table_bytes, active, mode) : run<16>(p, table_bytes, active, mode);
}

int main(int argc, char** argv)
{
    hipDeviceProp_t prop;
    if(hipGetDeviceProperties(&prop, 0) != hipSuccess) return 1;
    Probe p;
    p.cus = prop.multiProcessorCount;
    const size_t max_bytes = size_t(2048) << 20;
    if(hipMalloc(&p.table, max_bytes) != hipSuccess || hipMalloc(&p.sink, 64) != hipSuccess) return 1;
    if(hipMemset(p.table, 0, max_bytes) != hipSuccess) return 1;
    if(argc == 5)
    {
        const size_t mib = size_t(atoi(argv[1]));
        const int active = atoi(argv[2]), mode = atoi(argv[3]), bytes = atoi(argv[4]);
        if(mib < 1 || (mib << 20) > max_bytes || active < 1 || active > 64 || mode < 0 || mode > 2) return 2;
        printf("table %zu MiB active %d mode %d bytes %d: %.3f ns per wave-instruction per CU\n", mib, active, mode,
               bytes, run_bytes(p, mib << 20, active, mode, bytes));
    }
    else if(argc == 2 && strcmp(argv[1], "sizes") == 0)
    {
        printf("%s, %d CUs; random 64-B line per lane, dwordx4, ns per wave-instruction per CU\n", prop.gcnArchName, p.cus);
        printf("  table_MiB  active64  active16  active1\n");
        for(size_t mib: {1, 2, 4, 16, 64, 128, 192, 256, 384, 512, 1024, 2048})
            printf("  %9zu  %8.3f  %8.3f  %7.3f\n", mib, run<16>(p, mib << 20, 64, 0), run<16>(p, mib << 20, 16, 0),
                   run<16>(p, mib << 20, 1, 0));
    }
    else
    {
        printf("%s, %d CUs; ns per wave-level load instruction per CU (32 waves/CU, independent loads, 64 MiB table)\n",
               prop.gcnArchName, p.cus);
        const char* modes[] = {"random line per lane", "4 lanes per 64B line", "one address per wave"};
        for(int mode = 0; mode < 3; ++mode)
        {
            printf("mode: %s\n  active  dword   dwordx2 dwordx4\n", modes[mode]);
            for(int active: {64, 48, 32, 16, 8, 4, 1})
                printf("  %6d  %7.3f %7.3f %7.3f\n", active, run<4>(p, 64u << 20, active, mode),
                       run<8>(p, 64u << 20, active, mode), run<16>(p, 64u << 20, active, mode));
        }
    }
    (void)hipFree(p.table);
    (void)hipFree(p.sink);
    return 0;
}
