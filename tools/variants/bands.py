# variant: the number of XCD bands a walk queue is cut into (env PTG_BANDS; default 1024)
import os
import sys
p = sys.argv[1] + "/pt_kernels.hip"
s = open(p).read()
a = "constexpr uint32_t kBands = 1024;"
assert a in s
open(p, "w").write(s.replace(a, "constexpr uint32_t kBands = %d;" % int(os.environ["PTG_BANDS"])))
