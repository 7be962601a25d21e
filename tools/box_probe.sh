#!/bin/bash
# What the GPU box's host offers the CPU baseline: sockets, cores, the CPU
# quota and affinity of this job, and how the reference's baseline_render
# scales with OpenMP threads on it (v3 build, frame 0, 1280x720 x 16 spp).
R=${GRAFT_REPO_ROOT:-$(pwd)}
echo "== lscpu"; lscpu | grep -E "Model name|Socket|Core\(s\) per|Thread\(s\) per|^CPU\(s\)|NUMA node\(s\)|MHz"
echo "== nproc $(nproc)"
echo "== cgroup cpu.max: $(cat /sys/fs/cgroup/cpu.max 2>/dev/null || echo n/a)"
python3 -c "import os; a=sorted(os.sched_getaffinity(0)); print('== affinity', len(a), a[:8], '...', a[-4:])"
EXE=$R/oracle/_ref/v3_1280x720_s16_b4/ref_pt
for T in ${PROBE_THREADS:-16 32 64}; do
  echo "== threads $T"
  OMP_NUM_THREADS=$T OMP_PROC_BIND=close OMP_PLACES=cores timeout -k 5 120 $EXE $R/assets baseline 0 /tmp/probe.bgra || echo "failed $?"
done
