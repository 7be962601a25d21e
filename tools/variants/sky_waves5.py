# variant: the sky pass at 5 waves per SIMD (VGPR cap 96) instead of 4
import sys
p = sys.argv[1] + "/pt_kernels.hip"
s = open(p).read()
a = "#define PTG_SKY_WAVES 4 "
assert a in s
open(p, "w").write(s.replace(a, "#define PTG_SKY_WAVES 5 "))
