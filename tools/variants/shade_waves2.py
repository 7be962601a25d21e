# variant: the certified surface pass compiled for 2 waves per SIMD instead of 3
import sys
p = sys.argv[1] + "/pt_kernels.hip"
s = open(p).read()
a = "#define PTG_SHADE_WAVES 3"
assert a in s
open(p, "w").write(s.replace(a, "#define PTG_SHADE_WAVES 2"))
