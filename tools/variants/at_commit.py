# variant: csrc/ as of a git commit (env PTG_AT, default HEAD) - device AND
# host sources (the packer's block format must match the walker that reads
# it) - the "before" side of an A/B of uncommitted changes.  Writes
# .rebuild_host so tools/variant_build.sh compiles the host objects from
# these sources too.
import os
import subprocess
import sys
root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
rev = os.environ.get("PTG_AT", "HEAD")
pkg = "path-tracing...but-on-the-lumi-cluster_amd/csrc/"
files = subprocess.run(["git", "ls-tree", "-r", "--name-only", rev, pkg], cwd=root, capture_output=True, text=True,
                       check=True).stdout.split()
for f in files:
    src = subprocess.run(["git", "show", "%s:%s" % (rev, f)], cwd=root, capture_output=True, check=True).stdout
    dst = os.path.join(sys.argv[1], f[len(pkg):])
    os.makedirs(os.path.dirname(dst), exist_ok=True)
    open(dst, "wb").write(src)
open(os.path.join(sys.argv[1], ".rebuild_host"), "w").write(rev + "\n")
# entry points the current C ABI declares but the old sources lack: stubs (timing builds only)
p = os.path.join(sys.argv[1], "pt_kernels.hip")
s = open(p).read()
stubs = {"ptg_arith_selftest": 'extern "C" int ptg_arith_selftest(ptg_context*) { return -1; }   /* not available: never a passing self-test */',
         "ptg_tonemap_device": 'extern "C" int ptg_tonemap_device(ptg_context*, size_t, const ptg_float4*, ptg_uchar4*) { return -1; }',
         "ptg_set_chunk_paths": 'extern "C" int ptg_set_chunk_paths(ptg_context*, int) { return -1; }   /* not available */'}
for name, body in stubs.items():
    if name not in s:
        s += "\n" + body + "\n"
open(p, "w").write(s)
