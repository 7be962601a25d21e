#!/bin/bash
# Build and run the exhaustive div_by check (needs a gfx950 GPU).
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p "$R/gpurun_out"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -fno-fast-math -fhip-fp32-correctly-rounded-divide-sqrt \
  -I"$R/path-tracing...but-on-the-lumi-cluster_amd/csrc" "$R/tools/div_exhaustive.hip" -o "$R/gpurun_out/div_exhaustive"
timeout -k 10 120 "$R/gpurun_out/div_exhaustive"
