#!/bin/bash
# Calibrates the PMC counters the roofline uses on known access patterns:
# tools/_bin/ta_probe issues 32 waves/CU x 2048 wave-instructions per CU, each
# lane loading 16 B from its own random 64-B line (mode 0).  Separate --pmc
# passes (never combined with tracing).  Output: gpurun_out/probe_pmc/.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/probe_pmc
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
$R/tools/_bin/ta_probe sizes > $OUT/sizes.txt 2>&1 || exit 1
for CFG in "2 64 0 16" "64 64 0 16" "1024 64 0 16" "64 16 0 16" "64 64 1 16"; do
  TAG=$(echo $CFG | tr ' ' '_')
  for PASS in "TCP_TCC_READ_REQ_sum TCC_EA0_RDREQ_sum GRBM_GUI_ACTIVE" "TCC_HIT_sum TCC_MISS_sum" "SQ_INSTS_VMEM TA_BUSY_avr GRBM_GUI_ACTIVE" "FETCH_SIZE"; do
    NAME=$(echo $PASS | tr ' ' '_')
    timeout -s KILL 60 rocprofv3 --pmc $PASS --output-format csv -d $OUT/${TAG}_$NAME -o run -- $R/tools/_bin/ta_probe $CFG > $OUT/${TAG}_$NAME.log 2>&1 || { echo "pass $TAG $PASS failed"; tail -3 $OUT/${TAG}_$NAME.log; exit 1; }
  done
done
echo done
