# variant: 8-wide blocks (14 rows per block step) instead of 4-wide (7 rows);
# build with HOST_FLAGS=-DPTG_BLOCK_WIDTH=8 and hipcc -DPTG_BLOCK_WIDTH=8 (the
# packer and the walker must agree); the closest-hit walk capped at 128 VGPRs
import sys
p = sys.argv[1] + "/pt_kernels.hip"
s = open(p).read()
for a, b in (("#define PTG_WALK_WAVES 5", "#define PTG_WALK_WAVES 4"), ("#define PTG_SHADOW_WAVES 6", "#define PTG_SHADOW_WAVES 4")):
    assert a in s
    s = s.replace(a, b)
open(p, "w").write(s)
