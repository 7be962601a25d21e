# variant: the any-hit walk at wave priority PTG_ANYPRIO (env at patch time,
# default 1) below the closest-hit walk's 3 (the walks' s_setprio, k_wf_walk)
import os
import sys
p = sys.argv[1] + "/pt_kernels.hip"
s = open(p).read()
old = "    __builtin_amdgcn_s_setprio(3);\n    const uint32_t n = counts[2 * round + (ANY ? 1 : 0)];"
assert old in s
s = s.replace(old, "    __builtin_amdgcn_s_setprio(ANY ? %d : 3);\n    const uint32_t n = counts[2 * round + (ANY ? 1 : 0)];"
              % int(os.environ.get("PTG_ANYPRIO", "1")))
open(p, "w").write(s)
