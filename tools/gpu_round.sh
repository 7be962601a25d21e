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
    hazard) run pk_hazard 120 tools/_bin/pk_hazard; rc=$?; [ $rc -le 1 ] || exit $rc ;;
    anim) run gpu_anim 900 python -u -m pytest tests/test_gpu_animation.py -m gpu -x -v -s --timeout 880 --timeout-method thread || exit $? ;;
    slptri) run slp_tri_noslp 120 tools/_bin/slp_tri_noslp gpurun_out/slp_tri_noslp.bin || exit $?
            run slp_tri_slp 120 tools/_bin/slp_tri_slp gpurun_out/slp_tri_slp.bin || exit $?
            python3 tools/slp_tri_cmp.py gpurun_out/slp_tri_noslp.bin gpurun_out/slp_tri_slp.bin | tee gpurun_out/slp_tri_cmp.txt; rm -f gpurun_out/slp_tri_*.bin ;;
    slp) PTG_LIB=$P/ablate_slp/libptg.so run slp_rays 200 python tools/rays_diff.py || exit $? ;;
    slpvar) for v in ${SLPV:-slp}; do
              PTG_LIB=$P/ablate_$v/libptg.so run slp_rays_$v 200 python tools/rays_diff.py || exit $?
            done ;;
    slpbisect) for d in $P/ablate_slpT*; do
                 PTG_LIB=$d/libptg.so run slp_rays_$(basename $d) 200 python tools/rays_diff.py || exit $?
               done ;;
    tests) run gpu_tests 1100 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} || exit $? ;;
    debugtests) PTG_LIB=$P/ablate_debug/libptg.so run gpu_tests_ptg_debug 1100 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread --deselect tests/test_gpu_animation.py::test_every_frame_bit_identical_to_reference || exit $? ;;
    profile) run profile_${PROF_TAG:-r03} 1000 bash tools/profile_gpu.sh ${PROF_TAG:-r03} ${PROF_ARGS} || exit $? ;;
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit $? ;;
    exf64) run exhaustive_f64 1100 tools/exhaustive_f64.sh; rc=$?; [ $rc -le 1 ] || exit $rc ;;
    exf64bin) for fn in ${FNS:-0 1 2 3 4 5 6 7 8 9 10 11 12 13 14 15 16 17 18}; do
                run exhaustive_f64_$fn 600 tools/_bin/exhaustive_f64 $fn; rc=$?; [ $rc -le 1 ] || exit $rc
              done ;;
    parity) run gpu_parity 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_device_dropin.py -m gpu -x -q --timeout 500 --timeout-method thread || exit $? ;;
    ab) k=0
        for lib in ${LIBS:-default}; do
          k=$((k+1))   # run index: a library named twice (interleaved repeats) keeps both outputs
          for f in ${FRAMES:-0 450}; do
            if [ "$lib" = default ]; then L=""; else L=$P/ablate_$lib/libptg.so; fi
            PTG_LIB=$L run ab_${k}_${lib}_f$f 300 python tools/ablate.py --spp ${SPP:-1024} --frame $f --reps ${REPS:-2} ${ABARGS} || exit $?
          done
        done ;;
    bench) run bench 1100 python bench.py ${BENCH_ARGS} || exit $? ;;
    rehearse) run rehearse 1000 bash tools/rehearse.sh || exit $? ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo "== all steps done"
