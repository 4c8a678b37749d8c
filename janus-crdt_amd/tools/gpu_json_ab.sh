#!/bin/bash
# Fused JSON pass A: the wire-path and node GPU tests, then the json_apply leg with JANUS_JSON_FUSE=1 / 0 interleaved,
# and a kernel trace of each.  Usage: gpu_json_ab.sh <outdir>
set -o pipefail
OUT=${1:-gpurun_out/r05/json}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_json_gpu.py tests/test_node_gpu.py tests/test_apply_loop_gpu.py tests/test_shard_gpu.py -m gpu > "$OUT/pytest.log" 2>&1; rc=$?; tail -2 "$OUT/pytest.log"; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for f in 1 0; do
    JANUS_JSON_FUSE=$f timeout -k 10 200 python bench.py --workload json --steps 20 > "$OUT/b$f$i.json" 2>/dev/null || exit 1
    python3 -c "import json;d=json.loads(open('$OUT/b$f$i.json').read().strip().splitlines()[-1]);l=d['legs']['json_apply'];print('fuse', $f, l.get('ms_per_wave'), l.get('cold_wave_ms'))"
  done
done
for f in 1 0; do
  JANUS_JSON_FUSE=$f timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$OUT/kt$f" -o run --output-format csv -- python bench.py --workload json --steps 10 > "$OUT/kt$f.out" 2>&1 || exit 1
done
