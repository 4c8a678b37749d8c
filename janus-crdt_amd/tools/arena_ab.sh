#!/bin/bash
# A/B of the caller-arena legs on one box, interleaved: the one-shot arena (the caller's whole copy, then the wave)
# against the streamed one (jg_apply_stream_*) at each JANUS_ARENA_COPY_THREADS given.  ms_per_wave per run.
# Usage: arena_ab.sh <outdir> <rounds> <copiers>...
set -o pipefail
OUT=$1
ROUNDS=$2
shift 2
mkdir -p "$OUT"
B="janus-crdt_amd/build/bench_apply --accounts 1000000 --ops 1000000 --waves 3 --cpu-msgs 0 --device 0"
ms() { python3 -c "import json,sys; print(json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])['ms_per_wave'])" "$1"; }
for r in $(seq 1 "$ROUNDS"); do
    timeout -k 10 120 $B --arena > "$OUT/oneshot_$r.json" 2> "$OUT/oneshot_$r.err" || exit 1
    line="round $r: one-shot $(ms "$OUT/oneshot_$r.json")"
    for c in "$@"; do
        JANUS_ARENA_COPY_THREADS=$c timeout -k 10 120 $B --arena-stream > "$OUT/stream_${c}_$r.json" 2> "$OUT/stream_${c}_$r.err" || exit 1
        line="$line | streamed($c) $(ms "$OUT/stream_${c}_$r.json")"
    done
    echo "$line"
done
