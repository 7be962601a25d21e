#!/bin/bash
# ad-hoc timing sweep on the GPU box: tools/ab_run.sh "<env settings>" ... (one ablate.py run per setting)
set -e
FRAMES=${FRAMES:-"450 0"}
SPP=${SPP:-256}
for f in $FRAMES; do
 for e in "$@"; do
  echo "== $e frame $f"
  env $e timeout -k 10 200 python tools/ablate.py --spp $SPP --frame $f --reps 2 | grep -o '"wall_ms.*'
 done
done
