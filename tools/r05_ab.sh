#!/bin/bash
# Round-5 A/B session: the -m gpu suite on the default build, then 1024-spp
# timings of frames FR for each "label:lib:env" spec (best of REPS), then
# optionally the PTG_DEBUG suite (DEBUG=1).  Every GPU step has its own limit;
# the script stops at the first failure.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
P=path-tracing...but-on-the-lumi-cluster_amd/_build
if [ -z "$NOTESTS" ]; then
  echo "== gpu tests ($(date +%T))"
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/gpu_tests.txt 2>&1 || { tail -30 gpurun_out/gpu_tests.txt; exit 1; }
  tail -2 gpurun_out/gpu_tests.txt
fi
for spec in "$@"; do
  label=${spec%%:*}; rest=${spec#*:}; lib=${rest%%:*}; envs=${rest#*:}
  for f in ${FR:-0 450 1400}; do
    out=$(env $envs PTG_LIB=$P/$lib timeout -k 10 240 python tools/ablate.py --spp ${SPP:-1024} --frame $f --reps ${REPS:-2} --concurrency 2) || { echo "FAIL $label $f"; exit 1; }
    echo "$label f$f $(echo "$out" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d["wall_ms"], d["sha_bgra"][:12], json.dumps(d["kernels_ms"]))')"
  done
done | tee gpurun_out/ab.txt
if [ -n "$DEBUG" ]; then
  echo "== debug suite ($(date +%T))"
  PTG_LIB=$P/ablate_debug/libptg.so timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread --deselect tests/test_gpu_animation.py::test_every_frame_bit_identical_to_reference > gpurun_out/gpu_tests_ptg_debug.txt 2>&1 || { tail -30 gpurun_out/gpu_tests_ptg_debug.txt; exit 1; }
  tail -2 gpurun_out/gpu_tests_ptg_debug.txt
fi
