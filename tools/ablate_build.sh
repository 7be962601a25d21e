#!/bin/bash
# Timing-ablation builds (never parity builds): libptg.so variants with extra
# -D flags, written to <pkg>/_build/ablate_<tag>/libptg.so.  Select one at run
# time with PTG_LIB=<path> (native.py).
# Usage: tools/ablate_build.sh <tag> <extra hipcc flags, e.g. -fslp-vectorize> [...]
set -e
TAG=$1; shift
R=$(cd "$(dirname "$0")/.." && pwd)
PKG="$R/path-tracing...but-on-the-lumi-cluster_amd"
make -s -C "$PKG/csrc" >/dev/null
OUT="$PKG/_build/ablate_$TAG"
mkdir -p "$OUT"
cd "$PKG/csrc"
/opt/rocm/bin/hipcc -std=c++17 -O3 -fPIC --offload-arch=gfx950 -ffp-contract=off -fno-fast-math \
  -fhip-fp32-correctly-rounded-divide-sqrt -fno-slp-vectorize -I"$R/include" -I. "$@" -c pt_kernels.hip -o "$OUT/pt_kernels.o"
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o "$OUT/libptg.so" "$PKG"/_build/obj/{mesh_loader,bvh_builder,host_trace,scene,block_bvh}.o "$OUT/pt_kernels.o" -pthread
echo "$OUT/libptg.so"
