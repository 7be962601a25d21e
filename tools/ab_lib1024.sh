# ad-hoc: 1024-spp timings of libraries (PTG_LIB paths under the package's _build), frames FR
set -o pipefail
P=path-tracing...but-on-the-lumi-cluster_amd/_build
for lib in "$@"; do
 for f in ${FR:-0 450}; do
   echo "== $lib frame $f spp 1024"
   PTG_LIB=$P/$lib timeout -k 10 300 python tools/ablate.py --spp 1024 --frame $f --reps ${REPS:-2} --concurrency 2 | grep -o '"wall_ms.*'
 done
done
