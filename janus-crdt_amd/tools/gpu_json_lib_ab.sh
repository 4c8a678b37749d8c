#!/bin/bash
# Two builds of the library A/B on one box (JANUS_GPU_LIB): the json_apply leg interleaved, then one FETCH_SIZE
# and one WRITE_SIZE pass of each.  Usage: gpu_json_lib_ab.sh <outdir> <lib A> <lib B>
set -o pipefail
OUT=${1:-gpurun_out/r05/jsonlib}
A=${2:?lib A}
B=${3:?lib B}
mkdir -p "$OUT"
export TMPDIR=/tmp
for i in 1 2 3; do
  for v in A B; do
    lib=$A; [ $v = B ] && lib=$B
    JANUS_GPU_LIB=$lib timeout -k 10 200 python bench.py --workload json --steps 20 --no-cpu-baseline > "$OUT/b$v$i.json" 2>/dev/null || exit 1
    python3 -c "import json;d=json.loads(open('$OUT/b$v$i.json').read().strip().splitlines()[-1]);l=d['legs']['json_apply'];print('$v', l.get('ms_per_wave'), l.get('cold_wave_ms'))"
  done
done
for v in A B; do
  lib=$A; [ $v = B ] && lib=$B
  for C in FETCH_SIZE WRITE_SIZE; do
    JANUS_GPU_LIB=$lib timeout -s KILL 120 rocprofv3 --pmc $C -d "$OUT/pmc_${v}_$C" -o run --output-format csv -- python3 bench.py --steps 4 --warmup 1 --no-cpu-baseline --workload json > "$OUT/pmc_${v}_$C.out" 2>&1 || exit 1
  done
done
echo ab-done
