# variant: walk grid of 4 blocks per CU (all the LDS holds) instead of 3
import sys
p = sys.argv[1] + "/pt_kernels.hip"
s = open(p).read()
a = "constexpr uint32_t kWalkBlocksPerCu = 3;"
assert a in s
open(p, "w").write(s.replace(a, "constexpr uint32_t kWalkBlocksPerCu = 4;"))
