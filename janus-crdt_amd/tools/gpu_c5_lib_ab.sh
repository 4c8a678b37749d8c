#!/bin/bash
# Two library builds A/B on one box for the C5 apply loop from page-locked payloads (bench_apply --direct): A =
# LD_LIBRARY_PATH=<dir A> (overrides the binaries' RUNPATH), B = the in-tree lib; then a kernel trace of each.
# Usage: gpu_c5_lib_ab.sh <outdir> <lib dir A> [reps]
set -o pipefail
OUT=${1:-gpurun_out/r05/c5lib}
A=${2:?lib dir A}
N=${3:-3}
mkdir -p "$OUT"
export TMPDIR=/tmp
L="janus-crdt_amd/build/bench_apply --accounts 1000000 --ops 1000000 --waves 3 --cpu-msgs 0 --device 0 --direct"
for i in $(seq 1 $N); do
  LD_LIBRARY_PATH=$A timeout -k 10 120 $L > "$OUT/A$i.json" 2> "$OUT/A$i.err" || exit 1
  timeout -k 10 120 $L > "$OUT/B$i.json" 2> "$OUT/B$i.err" || exit 1
  python3 -c "
import json
for v in ('A','B'):
    d=json.loads(open('$OUT/'+v+'$i.json').read().strip().splitlines()[-1]); print(v, d['ms_per_wave'])"
done
LD_LIBRARY_PATH=$A timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$OUT/ktA" -o run --output-format csv -- $L > "$OUT/ktA.out" 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$OUT/ktB" -o run --output-format csv -- $L > "$OUT/ktB.out" 2>&1 || exit 1
python3 - "$OUT" <<'PY'
import csv, glob, sys
for v in "AB":
    f = glob.glob(f"{sys.argv[1]}/kt{v}/**/run_kernel_stats.csv", recursive=True)[0]
    for r in csv.DictReader(open(f)):
        if any(k in r["Name"] for k in ("k_resolve_rows", "k_scan<", "k_apply_emit", "k_track_insert")):
            print(v, r["Name"][:40], r["Calls"], round(float(r["AverageNs"]) / 1e3, 1), "us avg")
PY
