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
if "ptg_arith_selftest" not in s:
    s += '\nextern "C" int ptg_arith_selftest(ptg_context*) { return 0; }\n'
    open(p, "w").write(s)
