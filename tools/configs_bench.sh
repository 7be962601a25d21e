#!/bin/bash
# BASELINE configs 2-4 on one GPU (bench.py --config N), one line each in gpurun_out/config<N>.txt
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out
timeout -k 10 400 python bench.py --config 2 --steps 2 --warmup 1 --no-cpu-baseline --no-frame-setup --heavy-frame -1 --animation 0 > gpurun_out/config2.txt 2>&1 || exit $?
timeout -k 10 500 python bench.py --config 3 --steps 1 --warmup 1 --no-cpu-baseline --no-frame-setup --heavy-frame -1 > gpurun_out/config3.txt 2>&1 || exit $?
timeout -k 10 600 python bench.py --config 4 --steps 1 --warmup 0 --no-cpu-baseline --no-frame-setup > gpurun_out/config4.txt 2>&1 || exit $?
echo done
