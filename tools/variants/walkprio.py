# variant: the walk waves at a raised wave priority (s_setprio PRIO, env, default 2):
# when a walk wave and a shade / sky wave are both ready on a SIMD, the walk
# (latency-bound) issues first
import os, sys
p = sys.argv[1] + "/pt_kernels.hip"
s = open(p).read()
a = """                                                    unsigned long long* __restrict__ wstats)
{
    const uint32_t n = counts[2 * round + (ANY ? 1 : 0)];"""
assert a in s
s = s.replace(a, a.replace("{\n", "{\n    __builtin_amdgcn_s_setprio(%s);\n" % os.environ.get("PRIO", "2"), 1))
open(p, "w").write(s)
