# variant: camera_walk.py with the camera walk (round 0) compiled for 4 waves
# per SIMD (128 VGPRs: no spills) instead of 5 (96 VGPRs, 27 VGPRs spilled)
import os
import runpy
import sys
runpy.run_path(os.path.join(os.path.dirname(os.path.abspath(__file__)), "camera_walk.py"), run_name="__main__")
p = sys.argv[1] + "/pt_kernels.hip"
s = open(p).read()
old = "#define PTG_WALK_ATTR __attribute__((amdgpu_waves_per_eu(ANY ? PTG_SHADOW_WAVES : PTG_WALK_WAVES, 8)))"
assert old in s
s = s.replace(old, "#define PTG_WALK_ATTR __attribute__((amdgpu_waves_per_eu(ANY ? PTG_SHADOW_WAVES : (CAM ? 4 : PTG_WALK_WAVES), 8)))")
open(p, "w").write(s)
