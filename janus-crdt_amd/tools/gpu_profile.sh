#!/bin/bash
# Profile the bench on the GPU box: kernel trace + stats, then one PMC pass per counter group
# (FETCH_SIZE and WRITE_SIZE do not fit one pass on gfx950), then the per-launch HBM byte summary.
# Usage: gpu_profile.sh <outdir> [round label]
set -o pipefail
OUT=${1:-gpurun_out/prof}
LABEL=${2:-r02}
export TMPDIR=/tmp
mkdir -p "$OUT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- \
    python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --workload pnc-orset > "$OUT/bench_trace.json" || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace_exch" -o run --output-format csv -- \
    python3 bench.py --steps 16 --warmup 2 --no-cpu-baseline --workload exchange > "$OUT/bench_trace_exch.json" || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace_digest" -o run --output-format csv -- \
    python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --workload digest > "$OUT/bench_trace_digest.json" || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace_json" -o run --output-format csv -- \
    python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --workload json > "$OUT/bench_trace_json.json" || exit 1
for C in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 120 rocprofv3 --pmc $C -d "$OUT/pmc_$C" -o run --output-format csv -- \
        python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --workload pnc-orset > "$OUT/bench_pmc_$C.json" || exit 1
    timeout -s KILL 120 rocprofv3 --pmc $C -d "$OUT/pmc_exch_$C" -o run --output-format csv -- \
        python3 bench.py --steps 4 --warmup 1 --no-cpu-baseline --workload exchange > "$OUT/bench_pmc_exch_$C.json" || exit 1
    timeout -s KILL 120 rocprofv3 --pmc $C -d "$OUT/pmc_json_$C" -o run --output-format csv -- \
        python3 bench.py --steps 4 --warmup 1 --no-cpu-baseline --workload json > "$OUT/bench_pmc_json_$C.json" || exit 1
done
python3 janus-crdt_amd/tools/pmc_summary.py "$OUT" "$OUT/pmc_$LABEL.json" "$LABEL" || exit 1
echo profile-done
