#!/bin/bash
# Build and run the exhaustive checks of ref_math.h's exact fast paths (needs a gfx950 GPU).
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p "$R/gpurun_out"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -fno-fast-math -fhip-fp32-correctly-rounded-divide-sqrt \
  -I"$R/path-tracing...but-on-the-lumi-cluster_amd/csrc" "$R/tools/exhaustive.hip" -o "$R/gpurun_out/exhaustive"
timeout -k 10 300 "$R/gpurun_out/exhaustive"
