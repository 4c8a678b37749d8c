#!/bin/bash
# Copy a gpu_profile.sh run (gpurun_out/<dir>) into profiles/<round>/ (tracked): every leg's rocprofv3 kernel
# stats, the PMC counter passes and their per-launch summary (also profiles/pmc_<round>.json, which bench.py
# reads for roofline.traffic, the JSON VALU roofline and the OR-Set loop's decode bound), and the bench line of
# the same lease when the run made one.  Usage: collect_profile.sh <gpurun_out dir> <round>
set -e
SRC=${1:-gpurun_out/prof}
R=${2:-r04}
DST=profiles/$R
mkdir -p "$DST"
for leg in trace:bench trace_exch:exchange trace_digest:digest trace_json:json trace_apply:apply_loop trace_orset_loop:orset_loop; do
    cp "$SRC/${leg%%:*}/run_kernel_stats.csv" "$DST/kernel_stats_${leg##*:}.csv"
done
for p in pmc_FETCH_SIZE pmc_WRITE_SIZE pmc_exch_FETCH_SIZE pmc_exch_WRITE_SIZE pmc_json_FETCH_SIZE pmc_json_WRITE_SIZE \
         pmc_orset_loop_FETCH_SIZE pmc_orset_loop_WRITE_SIZE sq_json sq2_json sq_orset_loop sq2_orset_loop tcc_orset_loop; do
    [ -f "$SRC/$p/run_counter_collection.csv" ] && cp "$SRC/$p/run_counter_collection.csv" "$DST/$p.csv"
done
cp "$SRC/pmc_$R.json" "profiles/pmc_$R.json"
# the bench line (its last stdout line) and the kernel statistics of the same, traced process
[ -f "$SRC/bench_final.json" ] && tail -1 "$SRC/bench_final.json" > "$DST/bench_final.json"
[ -f "$SRC/trace_final/run_kernel_stats.csv" ] && cp "$SRC/trace_final/run_kernel_stats.csv" "$DST/kernel_stats_bench_final.csv"
[ -f "$SRC/bench_final_untraced.json" ] && tail -1 "$SRC/bench_final_untraced.json" > "$DST/bench_final_untraced.json"
echo "collected into $DST"
