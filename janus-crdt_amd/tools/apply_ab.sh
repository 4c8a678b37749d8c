#!/bin/bash
# Dev (GPU box): alternated A/B of two bench_apply builds (OLD=janus-crdt_amd/build/bench_apply_old).
O=$GRAFT_REPO_ROOT/gpurun_out/ab
mkdir -p $O
for r in 1 2 3 4; do
  timeout -k 10 200 ./janus-crdt_amd/build/bench_apply_old --waves 3 --cpu-msgs 0 > $O/old_$r.json 2>/dev/null || exit 1
  timeout -k 10 200 ./janus-crdt_amd/build/bench_apply --waves 3 --cpu-msgs 0 > $O/new_$r.json 2>/dev/null || exit 1
done
echo ab-done
