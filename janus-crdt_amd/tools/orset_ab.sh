#!/bin/bash
# Dev (GPU box): alternated OR-Set apply-loop runs, the build in janus-crdt_amd/abold (lib + bench) vs the tree's.
O=$GRAFT_REPO_ROOT/gpurun_out/oab
mkdir -p $O
for r in 1 2 3; do
  timeout -k 10 200 ./janus-crdt_amd/abold/build/bench_orset --sets 2000 --msgs 200000 --waves 3 --cpu-msgs 0 > $O/old_$r.json 2>/dev/null || exit 1
  timeout -k 10 200 ./janus-crdt_amd/build/bench_orset --sets 2000 --msgs 200000 --waves 3 --cpu-msgs 0 > $O/new_$r.json 2>/dev/null || exit 1
done
echo oab-done
