# ad-hoc: full GPU parity of an ablation library (PTG_LIB), then its timings
set -o pipefail
mkdir -p gpurun_out
P=path-tracing...but-on-the-lumi-cluster_amd/_build
LIB=$1; shift
PTG_LIB=$P/$LIB timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/parity_ab.txt 2>&1 || { tail -30 gpurun_out/parity_ab.txt; exit 1; }
tail -1 gpurun_out/parity_ab.txt
bash tools/ab1.sh "$@"
