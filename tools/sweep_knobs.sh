#!/bin/bash
# Timing sweeps on the GPU box.  Output: gpurun_out/sweep_knobs.log
#   default: per-kernel device times with every kernel on one stream
#            (concurrency 0) next to the default two-pipeline schedule
#   args:    env settings for tools/ab_run.sh (runtime knobs, no rebuild), e.g.
#            "PTG_CHUNK_LOG2=27" "PTG_SHADOW_RESIDENT=5" "PTG_WALK_OVERSUB=2"
set -o pipefail
mkdir -p gpurun_out
if [ $# -gt 0 ]; then
  FRAMES=${FRAMES:-"0 450"} SPP=${SPP:-1024} bash tools/ab_run.sh "$@" > gpurun_out/sweep_knobs.log 2>&1
  exit $?
fi
for f in 0 450; do
  for c in 0 2; do
    echo "== concurrency $c frame $f"
    timeout -k 10 200 python tools/ablate.py --spp 1024 --frame $f --reps 2 --concurrency $c | grep -o '"wall_ms.*' || exit 1
  done
done > gpurun_out/sweep_knobs.log 2>&1
