#!/bin/bash
# Rehearses bench.py's N>1 code paths on the one GPU of a test box: 2 ranks
# under torch.distributed.run sharing the device, gloo instead of RCCL
# (PTG_BENCH_REHEARSE=1; RCCL cannot put two ranks on one GPU), one run per
# shard mode.  Small frames; never a measurement.  Output: gpurun_out/rehearse_*.txt
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
port=29533
for mode in frames tiles samples; do
  port=$((port + 1))
  PTG_BENCH_REHEARSE=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port $port bench.py --gpus 2 --steps 2 --warmup 1 --width 640 --height 360 \
    --spp 64 --heavy-frame -1 --animation 2 --no-cpu-baseline --no-frame-setup --no-roofline --shard $mode \
    > gpurun_out/rehearse_$mode.txt 2>&1 || { echo "rehearse $mode failed"; tail -20 gpurun_out/rehearse_$mode.txt; exit 1; }
  grep '^{' gpurun_out/rehearse_$mode.txt | python3 -c "
import json, sys
d = json.loads(sys.stdin.read())
print('$mode', d['n_gpus'], d['scaling'], d['ranks']['world_size'], d['ranks']['backend'], d['ranks']['distinct_gpus'],
      [x['pci'] for x in d['ranks']['devices']], d['per_rank_seconds'])"
done
# bench.py launching its own ranks (no external launcher):
# the weak (frames) value plus the strong tile sub-record in one line
PTG_BENCH_REHEARSE=1 timeout -k 10 400 python3 bench.py --gpus 2 --steps 2 --warmup 1 --width 640 --height 360 \
  --spp 64 --heavy-frame -1 --animation 2 --no-cpu-baseline --no-frame-setup --no-roofline \
  > gpurun_out/rehearse_self.txt 2>&1 || { echo "rehearse self-launch failed"; tail -20 gpurun_out/rehearse_self.txt; exit 1; }
grep '^{' gpurun_out/rehearse_self.txt | python3 -c "
import json, sys
d = json.loads(sys.stdin.read())
print('self-launch', d['n_gpus'], d['scaling'], d['ranks']['world_size'], d['ranks']['backend'], d['ranks']['distinct_gpus'],
      'weak', d['value'], 'strong', d['strong']['value'], d['per_rank_seconds'], d['summary'])"
