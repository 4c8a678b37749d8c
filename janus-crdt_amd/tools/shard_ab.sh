#!/bin/bash
# Dev (GPU box): one rank of an 8-way key-space shard of the C5 apply loop, janus-crdt_amd/abold vs the tree's build.
O=$GRAFT_REPO_ROOT/gpurun_out/shab
mkdir -p $O
for r in 1 2 3; do
  for v in old new; do
    B=./janus-crdt_amd/build; [ $v = old ] && B=./janus-crdt_amd/abold/build
    timeout -k 10 200 $B/bench_apply --waves 3 --cpu-msgs 0 --rank 3 --world 8 > $O/${v}_$r.json 2>/dev/null || exit 1
  done
done
echo shab-done
