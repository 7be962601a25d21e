#!/bin/bash
# PMC passes over the wavefront kernels (run on the GPU box via gpurun).
# Usage: tools/profile_wf.sh <tag> [ablate.py args...]
set -o pipefail
TAG=${1:-wf}; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/prof_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
ARGS="$*"
W="$R/tools/ablate.py --spp 64 --reps 1 $ARGS"
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 $W > $OUT/trace.log 2>&1 || { echo "trace pass failed"; tail -20 $OUT/trace.log; exit 1; }
for PASS in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM SQ_INSTS_SALU" \
            "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY" "TCP_TCC_READ_REQ_sum TCC_EA0_RDREQ_sum GRBM_GUI_ACTIVE" \
            "SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_INST_LEVEL_VMEM SQ_LEVEL_WAVES" \
            "SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_TRANS_F64" \
            "SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_CVT SQ_IFETCH SQ_ACTIVE_INST_ANY" \
            "TCP_TOTAL_CACHE_ACCESSES_sum TCP_CACHE_MISS_sum TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum"; do
  NAME=$(echo $PASS | tr ' ' '_')
  timeout -k 10 300 rocprofv3 --pmc $PASS --output-format csv -d $OUT/pmc_$NAME -o run -- python3 $W > $OUT/pmc_$NAME.log 2>&1 || { echo "pmc pass $PASS failed"; tail -5 $OUT/pmc_$NAME.log; }
done
echo done
