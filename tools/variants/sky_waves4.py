# variant: the certified sky pass at 4 waves per SIMD (its VGPR cap 128) instead of 5
import sys
p = sys.argv[1] + "/pt_kernels.hip"
s = open(p).read()
a = "#define PTG_SKY_WAVES 5 "
assert a in s
open(p, "w").write(s.replace(a, "#define PTG_SKY_WAVES 4 "))
