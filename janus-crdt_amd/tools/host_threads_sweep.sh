#!/bin/bash
# Dev (GPU box): the apply loops at several host worker counts (the box's cgroup grants 16 CPUs of time).
set -e
O=$GRAFT_REPO_ROOT/gpurun_out
for T in ${JG_THREADS:-8 12 14 16}; do
  for r in 1 2; do
    JANUS_HOST_THREADS=$T timeout -k 10 200 ./janus-crdt_amd/build/bench_apply --waves 3 --cpu-msgs 0 > $O/ht_apply_${T}_$r.log
    JANUS_HOST_THREADS=$T timeout -k 10 200 ./janus-crdt_amd/build/bench_orset --sets 2000 --msgs 200000 --waves 3 --cpu-msgs 0 > $O/ht_orset_${T}_$r.log
  done
done
