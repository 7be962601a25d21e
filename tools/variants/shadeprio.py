# variant: the shade waves at a raised wave priority (s_setprio PRIO, env, default 1)
import os, sys
p = sys.argv[1] + "/pt_kernels.hip"
s = open(p).read()
a = """    uint32_t* __restrict__ redo_count, unsigned long long* __restrict__ counters, unsigned long long* __restrict__ redo_tally)
{
"""
assert a in s
s = s.replace(a, a + "    __builtin_amdgcn_s_setprio(%s);\n" % os.environ.get("PRIO", "1"), 1)
open(p, "w").write(s)
