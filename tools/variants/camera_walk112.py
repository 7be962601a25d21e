# variant: camera_walk.py with the camera walk (round 0) its own kernel,
# capped at PTG_CAM_VGPRS (default 112) VGPRs, so three of its waves (336)
# leave a shade wave (160) room on a SIMD
import os
import runpy
import sys
runpy.run_path(os.path.join(os.path.dirname(os.path.abspath(__file__)), "camera_walk.py"), run_name="__main__")
p = sys.argv[1] + "/pt_kernels.hip"
s = open(p).read()


def sub(old, new, count=1):
    global s
    assert s.count(old) == count, (old, s.count(old))
    s = s.replace(old, new)


ARGS = """(DevScene sc, PathSoA S, uint32_t* __restrict__ counts,
                                                    uint32_t round, const uint32_t* __restrict__ list, TraceOut tr,
                                                    uint32_t nxcd, unsigned long long* __restrict__ counters,
                                                    unsigned long long* __restrict__ wstats, CamArgs cam)"""
sub("template<bool ANY, bool COUNT, bool CAM = false>\n__global__ __launch_bounds__(kBlock) PTG_WALK_ATTR void k_wf_walk" + ARGS,
    "template<bool ANY, bool COUNT, bool CAM>\n__device__ __forceinline__ void walk_body" + ARGS)
CALL = "(sc, S, counts, round, list, tr, nxcd, counters, wstats, cam)"
sub("// Shading of one round is split by what the paths will run.",
    "template<bool ANY, bool COUNT, bool CAM = false>\n__global__ __launch_bounds__(kBlock) PTG_WALK_ATTR void k_wf_walk" + ARGS +
    "\n{\n    walk_body<ANY, COUNT, false>" + CALL + ";\n}\n"
    "template<bool COUNT>\n__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_num_vgpr(%s))) void k_wf_walk_cam" % os.environ.get("PTG_CAM_VGPRS", "112")
    + ARGS + "\n{\n    walk_body<false, COUNT, true>" + CALL + ";\n}\n\n"
    "// Shading of one round is split by what the paths will run.")
sub("(k_wf_walk<false, true, true>)", "(k_wf_walk_cam<true>)")
sub("(k_wf_walk<false, false, true>)", "(k_wf_walk_cam<false>)")
open(p, "w").write(s)
