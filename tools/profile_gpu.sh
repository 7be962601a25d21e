#!/bin/bash
# rocprofv3 evidence for the bench workload (run on the GPU box via gpurun).
#   1. kernel trace + stats of `bench.py` with every kernel on one stream
#      (--concurrency 0): the per-launch times are those of the kernels alone,
#      the same measurement as the bench line's roofline.isolated
#   2. separate PMC passes (counters never combined with tracing domains)
# Usage: tools/profile_gpu.sh <tag> [bench args...]
set -o pipefail
TAG=${1:-r02}; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/prof_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
BENCH="$R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-frame-setup --animation 0 --heavy-frame -1 --concurrency 0 $*"
cd /tmp
if [ -z "$NO_TRACE" ]; then
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 $BENCH > $OUT/trace.log 2>&1 || { echo "trace pass failed"; tail -20 $OUT/trace.log; exit 1; }
fi
# PASSES (env): the PMC passes to run, ';'-separated (default: the roofline's seven)
DEFAULT_PASSES="FETCH_SIZE;WRITE_SIZE;TCC_HIT_sum TCC_MISS_sum;SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM SQ_INSTS_SALU;SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY;TCP_TCC_READ_REQ_sum TCC_EA0_RDREQ_sum GRBM_GUI_ACTIVE;TA_BUSY_avr TD_BUSY_avr GRBM_GUI_ACTIVE"
IFS=';' read -r -a PASSLIST <<< "${PASSES:-$DEFAULT_PASSES}"
for PASS in "${PASSLIST[@]}"; do
  NAME=$(echo $PASS | tr ' ' '_')
  timeout -k 10 300 rocprofv3 --pmc $PASS --output-format csv -d $OUT/pmc_$NAME -o run -- python3 $BENCH --no-roofline > $OUT/pmc_$NAME.log 2>&1 || { echo "pmc pass $PASS failed"; tail -5 $OUT/pmc_$NAME.log; exit 1; }
done
echo done
