#!/bin/bash
# counting-pass comparison of the head build and the working tree (frame 0, 64 spp)
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out
P=path-tracing...but-on-the-lumi-cluster_amd/_build
for lib in head default; do
  if [ $lib = default ]; then L=""; else L=$P/ablate_$lib/libptg.so; fi
  for f in 0 450; do
    PTG_LIB=$L timeout -k 10 200 python tools/ablate.py --spp 64 --frame $f --reps 2 --counters > gpurun_out/cnt_${lib}_f$f.txt 2>&1 || exit $?
    PTG_LIB=$L timeout -k 10 200 python tools/ablate.py --spp 64 --frame $f --reps 2 --concurrency 0 > gpurun_out/iso_${lib}_f$f.txt 2>&1 || exit $?
  done
done
echo done
