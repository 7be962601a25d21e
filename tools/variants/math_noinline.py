# variant: the certified double-precision helpers (ref_math.h) out of line
# (__noinline__): one copy of each ocml routine instead of one per call site;
# with atm_rolled.py's rolled atmosphere loops
import sys, runpy
sys.argv = [sys.argv[0], sys.argv[1]]
runpy.run_path(__file__.replace("math_noinline.py", "atm_rolled.py"), run_name="__main__")
p = sys.argv[1] + "/device/ref_math.h"
s = open(p).read()
n = 0
for f in ["acc_exp", "exp_times", "add_mul_pow", "div_mul_pow", "times_cos", "times_sin", "times_one_minus_div_pow"]:
    a = "template<class MP> PTG_D float %s(" % f
    n += s.count(a)
    s = s.replace(a, "template<class MP> __device__ __noinline__ float %s(" % f)
assert n == 7, n
open(p, "w").write(s)
