#!/bin/bash
# Producer path: its parity tests (tests/test_apply_loop_gpu.py), then bench_submit for both workloads with the
# phase trace.  Usage: gpu_producer_check.sh <outdir>
set -o pipefail
OUT=${1:-gpurun_out/r05/prod}
mkdir -p "$OUT"
timeout -k 10 700 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_apply_loop_gpu.py -m gpu > "$OUT/pytest.log" 2>&1; rc=$?; tail -1 "$OUT/pytest.log"; [ $rc -eq 0 ] || exit $rc
JANUS_TRACE_SUBMIT=1 timeout -k 10 200 janus-crdt_amd/build/bench_submit --workload pnc --keys 1000000 --ops 1000000 --waves 3 --cpu-ops 50000 --device 0 > "$OUT/pnc.json" 2> "$OUT/pnc.err" || exit 1
tail -n 2 "$OUT/pnc.err"
JANUS_TRACE_SUBMIT=1 timeout -k 10 200 janus-crdt_amd/build/bench_submit --workload orset --keys 2000 --ops 200000 --waves 3 --cpu-ops 20000 --device 0 > "$OUT/orset.json" 2> "$OUT/orset.err" || exit 1
tail -n 2 "$OUT/orset.err"
python3 - "$OUT" <<'PY'
import json, sys
for w in ("pnc", "orset"):
    d = json.loads(open(f"{sys.argv[1]}/{w}.json").read().strip().splitlines()[-1])
    print(w, d["ms_per_wave"], d["ops_per_s"], d["parity_vs_oracle"], d["cpu_baseline"]["ops_per_s"])
PY
