# counting A/B: per library and frame, the work counters and isolated kernel times (256 spp)
set -o pipefail
cd $GRAFT_REPO_ROOT
P=path-tracing...but-on-the-lumi-cluster_amd/_build
for f in ${FRAMES:-0 450}; do
  for lib in ${LIBS:-default nocand2}; do
    if [ "$lib" = default ]; then L=""; else L=$P/ablate_$lib/libptg.so; fi
    PTG_LIB=$L timeout -k 10 300 python tools/ablate.py --spp 256 --frame $f --reps 2 --counters --concurrency 0 > gpurun_out/cnt_${lib}_f$f.txt 2>&1 || exit $?
    tail -1 gpurun_out/cnt_${lib}_f$f.txt | cut -c1-300
  done
done
