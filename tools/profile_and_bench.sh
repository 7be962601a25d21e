#!/bin/bash
# One GPU session: rocprofv3 trace + the PMC passes of the bench workload
# (tools/profile_gpu.sh), summarised into profiles/<tag>/ on the box (so the
# bench's roofline reads this tree's own profile), copied to gpurun_out/, then
# the bench line.  Usage (GPU box): tools/profile_and_bench.sh <tag>
set -o pipefail
TAG=${1:-final}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
timeout -k 10 1000 bash tools/profile_gpu.sh $TAG > gpurun_out/profile_$TAG.txt 2>&1 || { tail -20 gpurun_out/profile_$TAG.txt; exit 1; }
python3 tools/summarize_prof.py gpurun_out/prof_$TAG $TAG > gpurun_out/summarize_$TAG.txt 2>&1 || { tail -20 gpurun_out/summarize_$TAG.txt; exit 1; }
mkdir -p gpurun_out/profiles_$TAG && cp -r profiles/$TAG/. gpurun_out/profiles_$TAG/
timeout -k 10 1100 python bench.py > gpurun_out/bench.txt 2>&1 || { tail -20 gpurun_out/bench.txt; exit 1; }
grep '^{' gpurun_out/bench.txt | tail -1 > gpurun_out/profiles_$TAG/bench_line.json
echo done
