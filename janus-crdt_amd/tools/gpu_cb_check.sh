#!/bin/bash
# OR-Set commit check: the OR-Set GPU tests, then the pinned OR-Set apply loop three times, once traced, and a
# kernel trace.  Usage: gpu_cb_check.sh <outdir>
set -o pipefail
OUT=${1:-gpurun_out/r05/cb}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_orset_wire_gpu.py tests/test_node_gpu.py -m gpu > "$OUT/pytest.log" 2>&1; rc=$?; tail -3 "$OUT/pytest.log"; [ $rc -eq 0 ] || exit $rc
L="janus-crdt_amd/build/bench_orset --sets 2000 --msgs 200000 --waves 3 --cpu-msgs 0 --device 0 --direct"
for i in 1 2 3; do timeout -k 10 120 $L > "$OUT/run$i.json" 2> "$OUT/run$i.err" || exit 1; python3 -c "import json;print(json.loads(open('$OUT/run$i.json').read().strip().splitlines()[-1])['ms_per_wave'])"; done
JANUS_TRACE_APPLY=1 JANUS_TRACE_MERGE=1 timeout -k 10 120 $L > /dev/null 2> "$OUT/trace.err" || exit 1
grep -E "apply device|commit_tables" "$OUT/trace.err"
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$OUT/kt" -o run --output-format csv -- $L > "$OUT/kt.out" 2>&1 || exit 1
