# variant: the atmosphere integrals' loops kept rolled (#pragma unroll 1):
# smaller shade / sky code (instruction-cache pressure), less ILP
import sys
p = sys.argv[1] + "/device/path_tracer.h"
s = open(p).read()
n = 0
for a in ["    for(int i = 0; i < PRIMARY_ITERATIONS; ++i)\n", "        for(int j = 0; j < SECONDARY_ITERATIONS; ++j)\n",
          "            for(int j = 0; j < SECONDARY_ITERATIONS; ++j)\n"]:
    n += s.count(a)
    s = s.replace(a, a.replace("for(", "_Pragma(\"unroll 1\") for(", 1))
assert n >= 4, n
open(p, "w").write(s)
