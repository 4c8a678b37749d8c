#!/bin/bash
# Two bench_submit builds A/B on one box (untraced, interleaved), then one traced run of each.
# Usage: gpu_producer_ab.sh <outdir> <binary A> <binary B> [reps]
set -o pipefail
OUT=${1:-gpurun_out/r05/prodab}
A=${2:?binary A}
B=${3:?binary B}
N=${4:-3}
mkdir -p "$OUT"
timeout -k 10 700 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_apply_loop_gpu.py -m gpu > "$OUT/pytest.log" 2>&1; rc=$?; tail -1 "$OUT/pytest.log"; [ $rc -eq 0 ] || exit $rc
for i in $(seq 1 $N); do
  for v in A B; do
    exe=$A; [ $v = B ] && exe=$B
    timeout -k 10 200 $exe --workload pnc --keys 1000000 --ops 1000000 --waves 3 --cpu-ops 20000 --device 0 > "$OUT/pnc_$v$i.json" 2> "$OUT/pnc_$v$i.err" || exit 1
    timeout -k 10 200 $exe --workload orset --keys 2000 --ops 200000 --waves 3 --cpu-ops 5000 --device 0 > "$OUT/orset_$v$i.json" 2> "$OUT/orset_$v$i.err" || exit 1
    python3 -c "
import json
for w in ('pnc','orset'):
    d=json.loads(open('$OUT/'+w+'_$v$i.json').read().strip().splitlines()[-1]); print('$v', w, d['ms_per_wave'], d['parity_vs_oracle'])"
  done
done
for v in A B; do
  exe=$A; [ $v = B ] && exe=$B
  JANUS_TRACE_SUBMIT=1 timeout -k 10 200 $exe --workload pnc --keys 1000000 --ops 1000000 --waves 3 --cpu-ops 20000 --device 0 > "$OUT/tpnc_$v.json" 2> "$OUT/tpnc_$v.err" || exit 1
done
echo ab-done
