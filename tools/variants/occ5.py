# variant: the any-hit walk at 5 waves per SIMD (VGPR cap 96) instead of 6
import sys
p = sys.argv[1] + "/pt_kernels.hip"
s = open(p).read()
a = "#define PTG_SHADOW_WAVES 6\n"
assert a in s
open(p, "w").write(s.replace(a, "#define PTG_SHADOW_WAVES 5\n"))
