# variant: the exact (MathExact) shading passes capped at 64 VGPRs (8 waves per SIMD), so their
# few waves find room beside the persistent certified kernels
import sys
p = sys.argv[1] + "/pt_kernels.hip"
s = open(p).read()
for a, b in [("amdgpu_waves_per_eu(MP::kFast ? PTG_SHADE_WAVES : 2, 8)", "amdgpu_waves_per_eu(MP::kFast ? PTG_SHADE_WAVES : 8, 8)"),
             ("amdgpu_waves_per_eu(MP::kFast ? PTG_SKY_WAVES : 4, 8)", "amdgpu_waves_per_eu(MP::kFast ? PTG_SKY_WAVES : 8, 8)")]:
    assert a in s, a
    s = s.replace(a, b)
open(p, "w").write(s)
