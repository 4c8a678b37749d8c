#!/bin/bash
# Dev (GPU box): where the C5 apply loop's host time goes — cgroup quota and throttling counters around
# bench_apply runs at several host worker counts, with the per-chunk wave trace.
O=$GRAFT_REPO_ROOT/gpurun_out/probe
mkdir -p $O
{ cat /sys/fs/cgroup/cpu.max; nproc; lscpu | grep -E 'Model name|NUMA|L3'; } > $O/host.txt 2>&1
for T in ${JG_THREADS:-4 8 14}; do
  cat /sys/fs/cgroup/cpu.stat > $O/cpustat_before_$T.txt 2>&1
  JANUS_TRACE_WAVE=1 JANUS_HOST_THREADS=$T timeout -k 10 200 ./janus-crdt_amd/build/bench_apply --waves 3 --cpu-msgs 0 > $O/apply_$T.json 2> $O/apply_$T.trace || exit 1
  cat /sys/fs/cgroup/cpu.stat > $O/cpustat_after_$T.txt 2>&1
done
echo probe-done
