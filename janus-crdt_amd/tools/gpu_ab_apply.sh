#!/bin/bash
# Interleaved A/B of one apply-loop bench binary on one box: gpu_ab_apply.sh <out> <ENV_A> <ENV_B> <rounds> <binary> <args...>
set -o pipefail
OUT=$1; A=$2; B=$3; R=$4; shift 4
mkdir -p "$OUT"
for i in $(seq 1 $R); do
  for v in A B; do
    if [ $v = A ]; then E=$A; else E=$B; fi
    env $E timeout -k 10 120 "$@" > "$OUT/$v$i.json" 2> "$OUT/$v$i.err" || exit 1
    python3 -c "import json;d=json.loads(open('$OUT/$v$i.json').read().strip().splitlines()[-1]);print('$v', '$E', d['ms_per_wave'], d.get('device_busy_ms_per_wave'))"
  done
done
