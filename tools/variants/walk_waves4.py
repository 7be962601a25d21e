# variant: the closest-hit walk compiled for 4 waves per SIMD (VGPR cap 128) instead of 5 (96)
import sys
p = sys.argv[1] + "/pt_kernels.hip"
s = open(p).read()
a = "#define PTG_WALK_WAVES 5\n"
assert a in s
open(p, "w").write(s.replace(a, "#define PTG_WALK_WAVES 4\n"))
