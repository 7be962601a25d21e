# diagnostic variant: record the first 64 values whose certificate failed at
# one site (CERT_SITE, default 6 = times_one_minus_div_pow) with r, bpdf, q;
# read with ptg_debug_cert_values (tools/cert_trace.py)
import sys, os
site = int(os.environ.get("CERT_SITE", "6"))
p = sys.argv[1] + "/device/ref_math.h"
s = open(p).read()
a = "struct MathExact {   // glibc's algorithms"
assert a in s
s = s.replace(a, """__device__ double g_cert_vals[64 * 4];
__device__ unsigned g_cert_n;
__device__ inline void cert_record(double a, double b, double c, double d)
{
    const unsigned k = atomicAdd(&g_cert_n, 1u);
    if(k < 64) { g_cert_vals[4 * k] = a; g_cert_vals[4 * k + 1] = b; g_cert_vals[4 * k + 2] = c; g_cert_vals[4 * k + 3] = d; }
}
""" + a)
# anchored on the site name: the statement `mp.check(<certain>, v, CS_TIMES_ONE_MINUS_DIV_POW);`
# (possibly over several lines), whatever its condition currently reads
import re
m = re.search(r"mp\.check\(([^;]*?), v,\s*CS_TIMES_ONE_MINUS_DIV_POW\);", s)
assert m, "certificate site CS_TIMES_ONE_MINUS_DIV_POW not found"
cond = " ".join(m.group(1).split())
s = s[:m.end()] + "\n    if(MP::kFast && !(%s)) cert_record(r, x, q, v);" % cond + s[m.end():]
open(p, "w").write(s)
p = sys.argv[1] + "/pt_kernels.hip"
s = open(p).read()
s += """
extern "C" int ptg_debug_cert_values(double* out, unsigned* n)
{
    if(hipMemcpyFromSymbol(out, HIP_SYMBOL(ptg::dm::g_cert_vals), sizeof(double) * 256) != hipSuccess) return -1;
    if(hipMemcpyFromSymbol(n, HIP_SYMBOL(ptg::dm::g_cert_n), sizeof(unsigned)) != hipSuccess) return -1;
    return 0;
}
"""
open(p, "w").write(s)
