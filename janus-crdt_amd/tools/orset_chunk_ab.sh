#!/bin/bash
# Dev (GPU box): OR-Set apply loop at several wave chunk sizes (JANUS_WAVE_CHUNK messages; "auto" = the
# library's byte-sized default), alternated.
O=$GRAFT_REPO_ROOT/gpurun_out/ochunk
mkdir -p $O
for r in 1 2 3; do
  for v in ${VALUES:-auto 80000 131072}; do
    if [ "$v" = auto ]; then
      timeout -k 10 200 ./janus-crdt_amd/build/bench_orset --sets 2000 --msgs 200000 --waves 3 --cpu-msgs 0 > $O/v${v}_$r.json 2>/dev/null || exit 1
    else
      JANUS_WAVE_CHUNK=$v timeout -k 10 200 ./janus-crdt_amd/build/bench_orset --sets 2000 --msgs 200000 --waves 3 --cpu-msgs 0 > $O/v${v}_$r.json 2>/dev/null || exit 1
    fi
  done
done
echo ochunk-done
