#!/bin/bash
# A/B of two bench_submit builds on one box, interleaved (PN-Counter then OR-Set legs as bench.py runs them):
# usage: submit_ab.sh <outdir> <rounds> <binary>...   prints ms_per_wave (mean / median) per run
set -o pipefail
OUT=$1; R=$2; shift 2
mkdir -p "$OUT"
for r in $(seq 1 "$R"); do
  for b in "$@"; do
    for w in pnc orset; do
      if [ $w = pnc ]; then a="--workload pnc --keys 1000000 --ops 1000000"; else a="--workload orset --keys 2000 --ops 200000"; fi
      n=$(basename "$b")_${w}_$r
      timeout -k 10 120 "$b" $a --cpu-ops 0 --waves 5 --device 0 > "$OUT/$n.json" 2> "$OUT/$n.err" || exit 1
      python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['ms_per_wave'], d['ms_per_wave_median'])" "$OUT/$n.json" "$n"
    done
  done
done
