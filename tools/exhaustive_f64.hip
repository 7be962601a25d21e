// Exhaustive proof that the device's double-precision library calls return
// the very doubles glibc returns, for every argument the hot path can give
// them.
//
// The reference calls exp / log / pow / sin / cos / sqrt on floats, and C++
// promotes those to the C double functions (math.hh imports only fmin/fmax
// as float overloads); the results are then rounded to float, or first added
// to a float accumulator in double (path_tracer.hh:483-484, 531, 553-560).
// Device code calls ocml's f64 routines (csrc/device/ref_math.h dexp, dlog,
// dpow, dsin, dcos, dsqrt).  Every argument those calls receive is a float
// widened to double - except the outer sqrt of inv_erf (math.hh:455-463),
// whose argument is a double difference; inv_erf is therefore checked as a
// whole function of its float argument over its whole domain.
//
// For every one of the 2^32 float bit patterns x the GPU evaluates the
// product's own device function, the host evaluates glibc's (the library the
// reference and the oracle link), and the two doubles must be the same bits
// (any NaN matches any NaN):
//   exp(x) log(x) sqrt(x)                              all x
//   sin(x) cos(x)        |x| < 105414350 (glibc_math.h's domain; the path: [0, 2 pi])
//   (float)sin(x), (float)cos(x), (float)exp(x)   fsin / fcos / fexp, ocml, all x, float result
//   pow(x, 5.0)                                       fresnel_att (:91-98)
//   pow(x, 0.25)                                      path-space regularisation (:735-737)
//   pow(x, 1.5)                                       Mie phase (:531)
//   pow(x, (double)(1.0f / 2.4f))                     tonemap sRGB curve (:760-764)
//   inv_erf(x), float result, |x| <= 1 - 1e-6         film jitter (:12-25)
// Usage (GPU box): tools/exhaustive_f64.sh -> gpurun_out/exhaustive_f64.txt
#include <hip/hip_runtime.h>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdint>
#include <cstring>
#include <mutex>
#include <thread>
#include <vector>
#include "device/path_tracer.h"

using namespace ptg::dm;

enum Fn { F_EXP, F_LOG, F_SIN, F_COS, F_SQRT, F_POW5, F_POW025, F_POW15, F_POWSRGB, F_INVERF, F_FSIN, F_FCOS, F_FEXP, F_DEXP, F_DSIN, F_DCOS, F_DPOW5, F_DPOW15, F_DPOW025, F_COUNT };
// F_D*: "distance" rows - ocml's double (the certified shading, ref_math.h) against glibc's: the
// largest distance in ulps over all float arguments, which must not exceed kMaxLibDist
static bool is_distance(int fn) { return fn >= F_DEXP; }
static const char* kNames[F_COUNT] = {"exp(x)", "log(x)", "sin(x), |x| < 105414350", "cos(x), |x| < 105414350",
                                      "sqrt(x)", "pow(x, 5.0)", "pow(x, 0.25)", "pow(x, 1.5)",
                                      "pow(x, (double)(1.0f / 2.4f))", "inv_erf(x), |x| <= 1 - 1e-6",
                                      "(float)sin(x) (fsin)", "(float)cos(x) (fcos)", "(float)exp(x) (fexp)",
                                      "distance ocml exp(x)", "distance ocml sin(x)", "distance ocml cos(x)",
                                      "distance ocml pow(x, 5.0)", "distance ocml pow(x, 1.5)", "distance ocml pow(x, 0.25)"};
constexpr float kErfLimit = 1.0f - 1e-6f;   // sample_gaussian's clamp (path_tracer.hh:12-17)
constexpr float kSinCosLimit = 105414350.0f;   // glibc's reduce_sincos range (s_sin.c)
static __host__ __device__ bool in_domain(int fn, float x)
{
    if(fn == F_INVERF) return x >= -kErfLimit && x <= kErfLimit;
    if(fn == F_SIN || fn == F_COS) return fabsf(x) < kSinCosLimit;
    return true;
}


__global__ void k_eval(int fn, uint64_t begin, uint32_t n, uint64_t* __restrict__ out)
{
    for(uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x)
    {
        const float x = __uint_as_float(uint32_t(begin + i));
        const double d = (double)x;
        double r = 0;
        switch(fn)
        {
        case F_EXP: r = dexp(d); break;
        case F_LOG: r = dlog(d); break;
        case F_SIN: r = dsin(d); break;
        case F_COS: r = dcos(d); break;
        case F_SQRT: r = dsqrt(d); break;
        case F_POW5: r = dpow(d, 5.0); break;
        case F_POW025: r = dpow(d, 0.25); break;
        case F_POW15: r = dpow(d, 1.5); break;
        case F_POWSRGB: r = dpow(d, (double)(1.0f / 2.4f)); break;
        case F_FSIN: r = (double)fsin(x); break;
        case F_FCOS: r = (double)fcos(x); break;
        case F_FEXP: r = (double)fexp(x); break;
        case F_DEXP: r = exp(d); break;
        case F_DSIN: r = sin(d); break;
        case F_DCOS: r = cos(d); break;
        case F_DPOW5: r = pow(d, 5.0); break;
        case F_DPOW15: r = pow(d, 1.5); break;
        case F_DPOW025: r = pow(d, 0.25); break;
        default: r = (x >= -kErfLimit && x <= kErfLimit) ? (double)ptg::dm::inv_erf(x) : 0.0; break;
        }
        out[i] = __double_as_longlong(r);
    }
}

// host: glibc, as the reference and the oracle call it
// sign() (math.hh:127-132): note that +0 == -0.0f, so both zeros give -0.0f
static float host_sign(float v)
{
    if(v < 0) return -1.0f;
    if(v > 0) return 1.0f;
    return v == -0.0f ? -0.0f : +0.0f;
}
static float host_inv_erf(float x)   // oracle/pt_oracle.c inv_erf (math.hh:455-463)
{
    const float ln1x2 = (float)log((double)(1 - x * x));
    const float a = 0.147f;
    const float p = 2.0f / ((float)3.14159265358979323846 * a);
    const float k = p + ln1x2 * 0.5f;
    const float k2 = k * k;
    const double inner = sqrt((double)(k2 - ln1x2 * (1.0f / a)));
    return (float)((double)host_sign(x) * sqrt(inner - (double)k));
}
static double host_eval(int fn, float x)
{
    const double d = (double)x;
    switch(fn)
    {
    case F_EXP: return exp(d);
    case F_LOG: return log(d);
    case F_SIN: return sin(d);
    case F_COS: return cos(d);
    case F_SQRT: return sqrt(d);
    case F_POW5: return pow(d, 5.0);
    case F_POW025: return pow(d, 0.25);
    case F_POW15: return pow(d, 1.5);
    case F_POWSRGB: return pow(d, (double)(1.0f / 2.4f));
    case F_FSIN: return (double)(float)sin(d);
    case F_FCOS: return (double)(float)cos(d);
    case F_FEXP: return (double)(float)exp(d);
    case F_DEXP: return exp(d);
    case F_DSIN: return sin(d);
    case F_DCOS: return cos(d);
    case F_DPOW5: return pow(d, 5.0);
    case F_DPOW15: return pow(d, 1.5);
    case F_DPOW025: return pow(d, 0.25);
    default: return (x >= -kErfLimit && x <= kErfLimit) ? (double)host_inv_erf(x) : 0.0;
    }
}

static uint64_t bits(double v)
{
    uint64_t u;
    memcpy(&u, &v, 8);
    return u;
}
// distance in ulps of two doubles (as adjacent doubles count 1); NaN vs number
// or opposite signs (zeros aside): "infinite"
static uint64_t ulp_distance(double a, double b)
{
    if(a != a || b != b) return (a != a && b != b) ? 0 : ~0ull;
    if(a == 0 && b == 0) return 0;
    const int64_t ia = int64_t(bits(a) & 0x7fffffffffffffffull), ib = int64_t(bits(b) & 0x7fffffffffffffffull);
    if((bits(a) >> 63) != (bits(b) >> 63)) return ~0ull;
    return uint64_t(ia > ib ? ia - ib : ib - ia);
}

int main(int argc, char** argv)
{
    const int threads = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
    const uint32_t chunk = 1u << 26;
    uint64_t* dev = nullptr;
    uint64_t* host = nullptr;
    if(hipMalloc(&dev, size_t(chunk) * 8) != hipSuccess || hipHostMalloc(&host, size_t(chunk) * 8) != hipSuccess)
    {
        printf("allocation failed\n");
        return 2;
    }
    int first_fn = 0, last_fn = F_COUNT;
    if(argc > 1) { first_fn = atoi(argv[1]); last_fn = first_fn + 1; }
    int status = 0;
    for(int fn = first_fn; fn < last_fn; ++fn)
    {
        const auto t0 = std::chrono::steady_clock::now();
        std::atomic<uint64_t> mismatch{0}, float_mismatch{0}, domain{0};
        std::mutex mu;
        uint64_t max_dist = 0;   // distance rows: largest |ulp distance|, at max_x
        uint32_t max_x = 0;
        std::vector<uint32_t> examples;
        for(uint64_t b = 0; b < (1ull << 32); b += chunk)
        {
            hipLaunchKernelGGL(k_eval, dim3(8192), dim3(256), 0, nullptr, fn, b, chunk, dev);
            if(hipMemcpy(host, dev, size_t(chunk) * 8, hipMemcpyDeviceToHost) != hipSuccess)
            {
                printf("kernel / copy failed\n");
                return 2;
            }
            std::vector<std::thread> pool;
            for(int t = 0; t < threads; ++t)
                pool.emplace_back([&, t] {
                    uint64_t mis = 0, fmis = 0, dom = 0, dmax = 0;
                    uint32_t dx = 0;
                    for(uint32_t i = uint32_t(uint64_t(chunk) * t / threads); i < uint32_t(uint64_t(chunk) * (t + 1) / threads); ++i)
                    {
                        const uint32_t u = uint32_t(b + i);
                        float x;
                        memcpy(&x, &u, 4);
                        if(!in_domain(fn, x)) continue;
                        ++dom;
                        const double want = host_eval(fn, x);
                        double got;
                        memcpy(&got, &host[i], 8);
                        if(bits(want) == bits(got) || (want != want && got != got)) continue;
                        ++mis;
                        if(is_distance(fn))
                        {
                            const uint64_t dd = ulp_distance(want, got);
                            if(dd > dmax) { dmax = dd; dx = u; }
                        }
                        const float fw = (float)want, fg = (float)got;
                        uint32_t uw, ug;
                        memcpy(&uw, &fw, 4);
                        memcpy(&ug, &fg, 4);
                        if(uw != ug && !(fw != fw && fg != fg)) ++fmis;   // float bits (signed zeros differ)
                        std::lock_guard<std::mutex> g(mu);
                        if(examples.size() < 16) examples.push_back(u);
                    }
                    mismatch += mis;
                    float_mismatch += fmis;
                    domain += dom;
                    std::lock_guard<std::mutex> g(mu);
                    if(dmax > max_dist) { max_dist = dmax; max_x = dx; }
                });
            for(std::thread& th: pool) th.join();
            if((b / chunk) % 16 == 15)
            {
                printf("  %s: %llu / 64 chunks, %llu mismatches so far\n", kNames[fn], (unsigned long long)(b / chunk + 1),
                       (unsigned long long)mismatch.load());
                fflush(stdout);
            }
        }
        const double secs = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        printf("%s over %llu float inputs: %llu double mismatches (%llu of them also after rounding to float), %.1f s\n",
               kNames[fn], (unsigned long long)domain.load(), (unsigned long long)mismatch.load(),
               (unsigned long long)float_mismatch.load(), secs);
        for(uint32_t u: is_distance(fn) ? std::vector<uint32_t>() : examples)
        {
            float x;
            memcpy(&x, &u, 4);
            const double want = host_eval(fn, x);
            const double d = (double)x;
            double got = 0;
            // re-evaluate this one input on the device for the report
            hipLaunchKernelGGL(k_eval, dim3(1), dim3(1), 0, nullptr, fn, uint64_t(u), 1u, dev);
            if(hipMemcpy(&got, dev, 8, hipMemcpyDeviceToHost) != hipSuccess) return 2;
            printf("  x = 0x%08x (%.9g): glibc %.17g (0x%016llx), device %.17g (0x%016llx)\n", u, d, want,
                   (unsigned long long)bits(want), got, (unsigned long long)bits(got));
        }
        if(is_distance(fn))
        {   // the bound the certified shading relies on (ref_math.h kMaxLibDist)
            float x;
            memcpy(&x, &max_x, 4);
            printf("%s: largest distance %llu ulps (x = 0x%08x, %.9g); bound kMaxLibDist = %u: %s\n", kNames[fn],
                   (unsigned long long)max_dist, max_x, (double)x, ptg::dm::kMaxLibDist,
                   max_dist <= ptg::dm::kMaxLibDist ? "holds" : "VIOLATED");
            if(max_dist > ptg::dm::kMaxLibDist) status = 1;
        }
        else if(mismatch.load())
            status = 1;
        fflush(stdout);
    }
    return status;
}
