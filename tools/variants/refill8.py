# variant: refill a walk wave once 8 lanes are idle (instead of 24)
import sys
p = sys.argv[1] + "/pt_kernels.hip"
s = open(p).read()
a = "constexpr int kRefillIdle = 24;"
assert a in s
open(p, "w").write(s.replace(a, "constexpr int kRefillIdle = 8;"))
