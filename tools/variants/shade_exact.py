# variant: the surface pass with glibc's algorithms directly (MathExactLds, no redo pass)
import sys
p = sys.argv[1] + "/pt_kernels.hip"
s = open(p).read()
a = "using ShadeMath = MathFast;"
assert a in s
open(p, "w").write(s.replace(a, "using ShadeMath = MathExactLds;"))
