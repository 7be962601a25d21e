# variant (timing only, not exact): the shading kernels' ocml double library without its
# rounding certificates - the speed the certified MathFast pass is measured against
import sys
p = sys.argv[1] + "/device/ref_math.h"
s = open(p).read()
a = "    PTG_D void check(bool certain, double, int site) { fail_mask |= certain ? 0u : 1u << site; }"
assert a in s, a
open(p, "w").write(s.replace(a, "    PTG_D void check(bool, double, int) {}"))
