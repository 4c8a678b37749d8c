#!/bin/bash
# Dev (GPU box): alternated C5 apply-loop runs at two host worker counts (JG_A, JG_B), cgroup throttling counters around each.
O=$GRAFT_REPO_ROOT/gpurun_out/tab
mkdir -p $O
for r in 1 2 3; do
  for T in ${JG_A:-14} ${JG_B:-16}; do
    grep nr_throttled /sys/fs/cgroup/cpu.stat > $O/thr_${T}_$r.before 2>&1
    JANUS_HOST_THREADS=$T timeout -k 10 200 ./janus-crdt_amd/build/bench_apply --waves 3 --cpu-msgs 0 > $O/t${T}_$r.json 2>/dev/null || exit 1
    grep nr_throttled /sys/fs/cgroup/cpu.stat > $O/thr_${T}_$r.after 2>&1
  done
done
echo tab-done
