# ad-hoc: parity of the default build, then walk timings (256 spp) for the libs/env settings below
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/parity.txt 2>&1 || { tail -30 gpurun_out/parity.txt; exit 1; }
tail -1 gpurun_out/parity.txt
P=path-tracing...but-on-the-lumi-cluster_amd/_build
for spec in "$@"; do
 lib=${spec%%:*}; envs=${spec#*:}
 for f in ${FR:-450 0}; do
  for c in ${CC:-0 2}; do
   echo "== $lib [$envs] frame $f conc $c"
   env $envs PTG_LIB=$P/$lib timeout -k 10 200 python tools/ablate.py --spp 256 --frame $f --reps 2 --concurrency $c | grep -o '"wall_ms.*'
  done
 done
done
