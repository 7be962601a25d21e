# variant: 12-entry LDS stack windows (128 B of LDS per walk lane instead of
# 160), so the LDS holds 5 walk blocks per CU; the walk grid takes WALK_BLOCKS
# (env, default 4) of them per CU
import os, sys
p = sys.argv[1] + "/device/path_tracer.h"
s = open(p).read()
a = "    static constexpr uint32_t kCap = 16;"
assert a in s
open(p, "w").write(s.replace(a, "    static constexpr uint32_t kCap = 12;"))
p = sys.argv[1] + "/pt_kernels.hip"
s = open(p).read()
for a, b in [("constexpr uint32_t kWalkResident = 4;", "constexpr uint32_t kWalkResident = 5;"),
             ("constexpr uint32_t kWalkBlocksPerCu = 3;", "constexpr uint32_t kWalkBlocksPerCu = %s;" % os.environ.get("WALK_BLOCKS", "4"))]:
    assert a in s, a
    s = s.replace(a, b)
open(p, "w").write(s)
