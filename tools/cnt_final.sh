#!/bin/bash
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out
for f in 0 450; do
  timeout -k 10 300 python tools/ablate.py --spp 64 --frame $f --reps 1 --counters > gpurun_out/cnt_final_f$f.txt 2>&1 || exit $?
done
echo done
