#!/bin/bash
# Walk-kernel counters for an A/B of libptg builds (run on the GPU box via
# gpurun): one frame at 256 spp, every kernel on one stream (concurrency 0),
# a kernel trace plus separate PMC passes per library.
# Usage: tools/profile_walk.sh <tag> <frame> <lib>...   (libs relative to _build/)
set -o pipefail
TAG=$1; FRAME=$2; shift 2
R=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
P=$R/path-tracing...but-on-the-lumi-cluster_amd/_build
cd /tmp
for lib in "$@"; do
  OUT=$R/gpurun_out/pw_${TAG}/$(echo $lib | tr '/' '_')
  mkdir -p $OUT
  CMD="$R/tools/ablate.py --spp 256 --frame $FRAME --reps 1 --concurrency 0"
  PTG_LIB=$P/$lib timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 $CMD > $OUT/trace.log 2>&1 || { echo "trace failed $lib"; tail -5 $OUT/trace.log; exit 1; }
  for PASS in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM" \
              "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT" \
              "TCC_HIT_sum TCC_MISS_sum TA_BUSY_avr GRBM_GUI_ACTIVE" \
              "TCP_TCC_READ_REQ_sum TCC_EA0_RDREQ_sum TD_BUSY_avr GRBM_GUI_ACTIVE"; do
    NAME=$(echo $PASS | tr ' ' '_' | cut -c1-60)
    PTG_LIB=$P/$lib timeout -s KILL 120 rocprofv3 --pmc $PASS --output-format csv -d $OUT/pmc_$NAME -o run -- python3 $CMD > $OUT/pmc_$NAME.log 2>&1 || echo "pmc pass failed ($lib): $PASS"
  done
done
echo done
