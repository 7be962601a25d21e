#!/bin/bash
# Kernel timeline of one bench-size frame (rocprofv3 kernel trace only), for
# tools/timeline.py.  Usage (GPU box): tools/timeline.sh <tag> [ablate.py args]
set -o pipefail
TAG=${1:-tl}; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/timeline_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT -o run -- python3 $R/tools/ablate.py --spp 1024 --reps 1 "$@" > $OUT/run.log 2>&1
