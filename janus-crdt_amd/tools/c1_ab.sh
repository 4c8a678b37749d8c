#!/bin/bash
# Dev (GPU box): alternated C1 (bench_c1) and C5 (bench_apply) runs, the build in janus-crdt_amd/abold vs the tree's.
O=$GRAFT_REPO_ROOT/gpurun_out/c1ab
mkdir -p $O
for r in 1 2 3; do
  for v in old new; do
    B=./janus-crdt_amd/build; [ $v = old ] && B=./janus-crdt_amd/abold/build
    timeout -k 10 200 $B/bench_c1 > $O/c1_${v}_$r.json 2>/dev/null || exit 1
    timeout -k 10 200 $B/bench_apply --waves 3 --cpu-msgs 0 > $O/c5_${v}_$r.json 2>/dev/null || exit 1
  done
done
echo c1ab-done
