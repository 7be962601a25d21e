# variant: csrc/ device sources as of a git commit (env PTG_AT, default HEAD) -
# the "before" side of an A/B of uncommitted changes
import os
import subprocess
import sys
root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
rev = os.environ.get("PTG_AT", "HEAD")
for f in ("device/path_tracer.h", "device/block_format.h", "device/wavefront.h", "device/ref_math.h", "pt_kernels.hip"):
    src = subprocess.run(["git", "show", "%s:path-tracing...but-on-the-lumi-cluster_amd/csrc/%s" % (rev, f)], cwd=root,
                         capture_output=True, check=True).stdout
    open(os.path.join(sys.argv[1], f), "wb").write(src)
# entry points the current C ABI declares but the old sources lack: stubs (timing builds only)
p = os.path.join(sys.argv[1], "pt_kernels.hip")
s = open(p).read()
stubs = {"ptg_arith_selftest": 'extern "C" int ptg_arith_selftest(ptg_context*) { return 0; }',
         "ptg_tonemap_device": 'extern "C" int ptg_tonemap_device(ptg_context*, size_t, const ptg_float4*, ptg_uchar4*) { return -1; }'}
for name, body in stubs.items():
    if name not in s:
        s += "\n" + body + "\n"
open(p, "w").write(s)
