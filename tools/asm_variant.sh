#!/bin/bash
# Diagnostic libptg.so variants built from the SLP-vectorised device assembly
# of pt_kernels.hip with chosen packed instructions of one kernel scalarised
# (tools/slp_scalarize.py).  Never a parity build of the shipped tree.
#   tools/asm_variant.sh <tag> <function label> <indices|all|none> [temp VGPR]
#   tools/asm_variant.sh <tag> - splice:<kernel label>[,...]   (those kernels from the -fno-slp-vectorize build)
# Output: <pkg>/_build/ablate_<tag>/libptg.so (select with PTG_LIB).
set -e
TAG=$1; FUNC=$2; WHICH=$3; TEMP=$4
R=$(cd "$(dirname "$0")/.." && pwd)
PKG="$R/path-tracing...but-on-the-lumi-cluster_amd"
BASE=/tmp/ptg_asm_base
DEVS=pt_kernels-hip-amdgcn-amd-amdhsa-gfx950.s
make -s -C "$PKG/csrc" >/dev/null
if [ ! -f $BASE/cmds.txt ]; then
  mkdir -p $BASE && cd $BASE
  /opt/rocm/bin/hipcc -### -std=c++17 -O3 -fPIC --offload-arch=gfx950 -ffp-contract=off -fno-fast-math \
    -fhip-fp32-correctly-rounded-divide-sqrt -fslp-vectorize -I"$R/include" -I"$PKG/csrc" -save-temps \
    -c "$PKG/csrc/pt_kernels.hip" -o pk.o 2> cmds_raw.txt
  grep '^ "' cmds_raw.txt > cmds.txt
  while read -r line; do eval "$line" 2>/dev/null; done < cmds.txt
  cp $DEVS $DEVS.orig
fi
W=$(mktemp -d /tmp/ptg_asmvar_XXXX)
cp $BASE/* $W/ && cd $W
if [ "$WHICH" = none ]; then cp $DEVS.orig $DEVS
elif [ "${WHICH#splice:}" != "$WHICH" ]; then
  [ -f $BASE/noslp.s ] || /opt/rocm/bin/hipcc -std=c++17 -O3 -fPIC --offload-arch=gfx950 --offload-device-only -ffp-contract=off \
    -fno-fast-math -fhip-fp32-correctly-rounded-divide-sqrt -fno-slp-vectorize -I"$R/include" -I"$PKG/csrc" -S \
    "$PKG/csrc/pt_kernels.hip" -o $BASE/noslp.s 2>/dev/null
  python3 "$R/tools/asm_splice.py" $DEVS.orig $BASE/noslp.s $DEVS "${WHICH#splice:}"
else python3 "$R/tools/slp_scalarize.py" $DEVS.orig $DEVS "$FUNC" "$WHICH" $TEMP; fi
sed -n '4,10p' cmds.txt | sed "s#/tmp/ptg_asm_base#$W#g" > steps.txt
while read -r line; do eval "$line" 2>/dev/null || { echo "step failed: ${line:0:120}"; exit 1; }; done < steps.txt
OUT="$PKG/_build/ablate_$TAG"
mkdir -p "$OUT"
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o "$OUT/libptg.so" "$PKG"/_build/obj/{mesh_loader,bvh_builder,host_trace,scene,block_bvh}.o $W/pk.o -pthread
cd / && rm -rf "$W"
echo "$OUT/libptg.so"
