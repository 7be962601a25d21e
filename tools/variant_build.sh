#!/bin/bash
# Timing/diagnostic variant of libptg.so built from a patched scratch copy of
# csrc/ (never a parity build of the shipped tree): tools/variant_build.sh
# <tag> <patch.py> [extra hipcc flags].  <patch.py> gets the scratch csrc
# directory as argv[1] and edits it.  Output: <pkg>/_build/ablate_<tag>/libptg.so,
# selected at run time with PTG_LIB.  HOST_FLAGS=...: host objects rebuilt with those flags.
set -e
TAG=$1; PATCH=$2; shift 2
R=$(cd "$(dirname "$0")/.." && pwd)
PKG="$R/path-tracing...but-on-the-lumi-cluster_amd"
make -s -C "$PKG/csrc" >/dev/null
W=$(mktemp -d /tmp/ptg_variant_XXXX)
cp -r "$PKG/csrc/." "$W/"
python3 "$PATCH" "$W"
OUT="$PKG/_build/ablate_$TAG"
mkdir -p "$OUT"
cd "$W"
/opt/rocm/bin/hipcc -std=c++17 -O3 -fPIC --offload-arch=gfx950 -ffp-contract=off -fno-fast-math \
  -fhip-fp32-correctly-rounded-divide-sqrt -fno-slp-vectorize -I"$R/include" -I. "$@" -c pt_kernels.hip -o "$OUT/pt_kernels.o"
HOST_OBJS=$(echo "$PKG"/_build/obj/{mesh_loader,bvh_builder,host_trace,scene,block_bvh}.o)
# the variant changes the host side too (e.g. -DPTG_BLOCK_WIDTH=8, or a whole
# commit's sources: at_commit.py writes .rebuild_host): rebuild it from the
# scratch copy, never mix the shipped packer with other walker sources
if [ -n "$HOST_FLAGS" ] || [ -f "$W/.rebuild_host" ]; then
  HOST_OBJS=""
  for f in mesh_loader bvh_builder host_trace scene block_bvh; do
    g++ -std=c++17 -O2 -fPIC -ffp-contract=off -fno-fast-math -I"$R/include" -I"$PKG/_gen" -I. -pthread $HOST_FLAGS \
      -c host/$f.cpp -o "$OUT/$f.o"
    HOST_OBJS="$HOST_OBJS $OUT/$f.o"
  done
fi
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o "$OUT/libptg.so" $HOST_OBJS "$OUT/pt_kernels.o" -pthread
rm -rf "$W"
echo "$OUT/libptg.so"
