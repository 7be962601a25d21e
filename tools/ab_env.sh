# ad-hoc: timings of the default library under environment settings (no parity run)
# usage: SPP=1024 FR="0 450" tools/ab_env.sh "X=1" "PTG_SLOTS=3" ...
set -o pipefail
mkdir -p gpurun_out
for envs in "$@"; do
 for f in ${FR:-0 450}; do
   echo "== [$envs] frame $f spp ${SPP:-1024}"
   env $envs timeout -k 10 300 python tools/ablate.py --spp ${SPP:-1024} --frame $f --reps ${REPS:-2} --concurrency 2 | grep -o '"wall_ms.*'
 done
done
