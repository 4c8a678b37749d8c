#!/bin/bash
# Interleaved A/B of the OR-Set apply loop from page-locked payloads on one box: gpu_ab_orset.sh <out> <ENV_A> <ENV_B> [rounds]
set -o pipefail
OUT=$1; A=$2; B=$3; R=${4:-4}
mkdir -p "$OUT"
L="janus-crdt_amd/build/bench_orset --sets 2000 --msgs 200000 --waves 3 --cpu-msgs 0 --device 0 --direct"
for i in $(seq 1 $R); do
  for v in A B; do
    if [ $v = A ]; then E=$A; else E=$B; fi
    env $E timeout -k 10 120 $L > "$OUT/$v$i.json" 2> "$OUT/$v$i.err" || exit 1
    python3 -c "import json;d=json.loads(open('$OUT/$v$i.json').read().strip().splitlines()[-1]);print('$v', '$E', d['ms_per_wave'], d['device_busy_ms_per_wave'])"
  done
done
