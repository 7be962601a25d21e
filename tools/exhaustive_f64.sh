#!/bin/bash
# Build and run tools/exhaustive_f64.hip (needs a gfx950 GPU): the device's f64
# exp/log/sin/cos/sqrt/pow and inv_erf against glibc on every float input.
# Output: gpurun_out/exhaustive_f64.txt.  Optional argument: one function index.
set -o pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p "$R/gpurun_out"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -fno-fast-math -fhip-fp32-correctly-rounded-divide-sqrt \
  -fno-slp-vectorize -I"$R/include" -I"$R/path-tracing...but-on-the-lumi-cluster_amd/csrc" "$R/tools/exhaustive_f64.hip" \
  -o "$R/gpurun_out/exhaustive_f64" -pthread || exit 2
timeout -k 10 1000 "$R/gpurun_out/exhaustive_f64" "$@" | tee "$R/gpurun_out/exhaustive_f64.txt"
