#!/bin/bash
# Profile the bench on the GPU box: kernel trace + stats of every bench leg, then one PMC pass per counter
# group (FETCH_SIZE and WRITE_SIZE do not fit one pass on gfx950; SQ_INSTS_VALU for the JSON leg's
# instruction roofline), then the per-launch HBM byte summary (pmc_summary.py).
# Usage: gpu_profile.sh <outdir> [round label]
set -o pipefail
OUT=${1:-gpurun_out/prof}
LABEL=${2:-r03}
export TMPDIR=/tmp
mkdir -p "$OUT"
trace() {  # trace <name> <seconds> <command...>
    local name=$1 secs=$2
    shift 2
    timeout -k 10 "$secs" rocprofv3 --kernel-trace --stats -d "$OUT/$name" -o run --output-format csv -- "$@" > "$OUT/$name.out" || exit 1
}
trace trace 300 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --workload pnc-orset
trace trace_exch 300 python3 bench.py --steps 16 --warmup 2 --no-cpu-baseline --workload exchange
trace trace_digest 300 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --workload digest
trace trace_json 300 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --workload json
trace trace_apply 300 janus-crdt_amd/build/bench_apply --accounts 1000000 --ops 1000000 --waves 3 --cpu-msgs 0 --device 0
trace trace_orset_loop 300 janus-crdt_amd/build/bench_orset --sets 2000 --msgs 200000 --waves 3 --cpu-msgs 0 --device 0
for C in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 120 rocprofv3 --pmc $C -d "$OUT/pmc_$C" -o run --output-format csv -- \
        python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --workload pnc-orset > "$OUT/bench_pmc_$C.json" || exit 1
    timeout -s KILL 120 rocprofv3 --pmc $C -d "$OUT/pmc_exch_$C" -o run --output-format csv -- \
        python3 bench.py --steps 4 --warmup 1 --no-cpu-baseline --workload exchange > "$OUT/bench_pmc_exch_$C.json" || exit 1
    timeout -s KILL 120 rocprofv3 --pmc $C -d "$OUT/pmc_json_$C" -o run --output-format csv -- \
        python3 bench.py --steps 4 --warmup 1 --no-cpu-baseline --workload json > "$OUT/bench_pmc_json_$C.json" || exit 1
done
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU -d "$OUT/sq_json" -o run --output-format csv -- \
    python3 bench.py --steps 4 --warmup 1 --no-cpu-baseline --workload json > "$OUT/bench_sq_json.json" || exit 1
python3 janus-crdt_amd/tools/pmc_summary.py "$OUT" "$OUT/pmc_$LABEL.json" "$LABEL" || exit 1
echo profile-done
