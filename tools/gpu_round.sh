#!/bin/bash
# One GPU-box session: the -m gpu suite, smoke, and optional extra steps.
# Every GPU step has its own time limit; the script stops at the first
# fault / abort / timeout (exit status >= 2 of a step, or of pytest != 0/1).
#   STEPS="probe slp tests smoke" tools/gpu_round.sh     (default: tests smoke)
#   PYTEST_K="expression"   deselect / select tests
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
export TMPDIR=/tmp
P=path-tracing...but-on-the-lumi-cluster_amd/_build
run() {   # run <name> <seconds> <cmd...>: output to gpurun_out/<name>.txt
  local name=$1 secs=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.txt" 2>&1
  local rc=$?
  tail -4 "gpurun_out/$name.txt"
  echo "== $name exit $rc"
  return $rc
}
for step in ${STEPS:-tests smoke}; do
  case $step in
    probe) run pk_probe 120 tools/_bin/pk_probe; rc=$?; [ $rc -le 1 ] || exit $rc ;;
    slp) PTG_LIB=$P/ablate_slp/libptg.so run slp_rays 200 python tools/rays_diff.py || exit $? ;;
    slpbisect) for d in $P/ablate_slpT*; do
                 PTG_LIB=$d/libptg.so run slp_rays_$(basename $d) 200 python tools/rays_diff.py || exit $?
               done ;;
    tests) run gpu_tests 1100 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} || exit $? ;;
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit $? ;;
    exf64) run exhaustive_f64 1100 tools/exhaustive_f64.sh; rc=$?; [ $rc -le 1 ] || exit $rc ;;
    bench) run bench 1100 python bench.py || exit $? ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo "== all steps done"
