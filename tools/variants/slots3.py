# variant: three concurrent wavefront chunk pipelines instead of two
import sys
p = sys.argv[1] + "/pt_kernels.hip"
s = open(p).read()
a = "constexpr uint32_t kWfSlots = 2;"
assert a in s
open(p, "w").write(s.replace(a, "constexpr uint32_t kWfSlots = 3;"))
