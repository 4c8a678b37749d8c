#!/bin/bash
# A/B of JSON pass A (k_scan) builds: for each library given, one PMC pass of the LDS counters over the json bench
# leg and one timed run of it, the k_scan sums printed per library.  Usage: json_lds_ab.sh <outdir> <lib.so>...
set -o pipefail
OUT=$1
shift
export TMPDIR=/tmp
mkdir -p "$OUT"
CTR=SQ_LDS_BANK_CONFLICT,SQ_LDS_IDX_ACTIVE,SQ_INSTS_LDS,SQ_WAVE_CYCLES
for LIB in "$@"; do
    name=$(basename "$LIB" .so)
    echo "[$(date +%H:%M:%S)] $name"
    JANUS_GPU_LIB=$PWD/$LIB timeout -s KILL 150 rocprofv3 --pmc $CTR -d "$OUT/$name" -o run --output-format csv -- \
        python3 bench.py --steps 4 --warmup 1 --no-cpu-baseline --workload json > "$OUT/$name.pmc.out" 2> "$OUT/$name.pmc.err" || exit 1
    JANUS_GPU_LIB=$PWD/$LIB timeout -k 10 150 python3 bench.py --steps 8 --warmup 2 --no-cpu-baseline --workload json \
        > "$OUT/$name.json" 2> "$OUT/$name.err" || exit 1
    python3 - "$OUT/$name" <<'EOF' || exit 1
import csv, glob, sys, collections
tot = collections.Counter()
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "k_scan<" in r.get("Kernel_Name", "") and "k_scan_slow" not in r["Kernel_Name"]:
            tot[r["Counter_Name"]] += float(r["Counter_Value"])
c, a = tot["SQ_LDS_BANK_CONFLICT"], tot["SQ_LDS_IDX_ACTIVE"]
print(sys.argv[1], {k: int(v) for k, v in tot.items()}, "conflict_frac", round(c / a, 4) if a else None)
EOF
    tail -c 400 "$OUT/$name.json"
    echo
done
