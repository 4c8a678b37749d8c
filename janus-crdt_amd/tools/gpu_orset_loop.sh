#!/bin/bash
# The OR-Set apply loop from page-locked payloads (bench_orset --direct, ORSetWorkload shape) on its own: three
# untimed-profiler runs for the wave time, a kernel trace with stats, and the counter passes pmc_summary.py's
# orset_loop() reads (one pass per counter group), then its per-kernel summary.  Usage: gpu_orset_loop.sh <outdir>
set -o pipefail
OUT=${1:-gpurun_out/orset_loop}
export TMPDIR=/tmp
mkdir -p "$OUT"
ORSET_LOOP="janus-crdt_amd/build/bench_orset --sets 2000 --msgs 200000 --waves 3 --cpu-msgs 0 --device 0 --direct"
SQ=SQ_INSTS_VALU,SQ_INSTS_SALU,SQ_INSTS_LDS,SQ_INSTS_VMEM,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_WAVE_CYCLES,SQ_BUSY_CYCLES
SQ2=SQ_ACTIVE_INST_ANY,SQ_LDS_BANK_CONFLICT,SQ_LDS_IDX_ACTIVE,SQ_WAIT_INST_LDS
TCC=TCC_ATOMIC_sum,TCC_HIT_sum,TCC_MISS_sum,TCC_EA0_RDREQ_sum
for i in 1 2 3; do
    timeout -k 10 120 $ORSET_LOOP > "$OUT/run$i.json" 2> "$OUT/run$i.err" || exit 1
done
JANUS_TRACE_APPLY=1 timeout -k 10 120 $ORSET_LOOP > "$OUT/run_trace.json" 2> "$OUT/run_trace.err" || exit 1  # the wave's setup / tail phases
echo "runs done"
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$OUT/trace_orset_loop" -o run --output-format csv -- $ORSET_LOOP > "$OUT/trace.out" 2>&1 || exit 1
echo "trace done"
pass() {  # pass <name> <counters>
    timeout -s KILL 150 rocprofv3 --pmc "$2" -d "$OUT/$1" -o run --output-format csv -- $ORSET_LOOP > "$OUT/$1.out" 2>&1 || exit 1
    echo "pass $1 done"
}
pass pmc_orset_loop_FETCH_SIZE FETCH_SIZE
pass pmc_orset_loop_WRITE_SIZE WRITE_SIZE
pass sq_orset_loop $SQ
pass sq2_orset_loop $SQ2
pass tcc_orset_loop $TCC
python3 - "$OUT" > "$OUT/summary.json" <<'PY' || exit 1
import json, sys
from pathlib import Path
sys.path.insert(0, "janus-crdt_amd/tools")
import pmc_summary as p
d = Path(sys.argv[1])
runs = [json.loads((d / f"run{i}.json").read_text().strip().splitlines()[-1]) for i in (1, 2, 3)]
k = p.orset_loop(d) or {}
print(json.dumps({"ms_per_wave": [r["ms_per_wave"] for r in runs], "kernels": k}, indent=1))
PY
python3 -c "
import json,sys; d=json.load(open('$OUT/summary.json')); print('ms_per_wave', d['ms_per_wave'])
for k,v in sorted(d['kernels'].items(), key=lambda kv: -(kv[1]['us_per_wave'] or 0))[:12]:
    print(f\"{k:28s} {v['us_per_wave'] or 0:8.1f} us  {v['hbm_bytes_per_wave_random_lines']/1e9:6.3f} GB  hit {v['tcc_hit_rate'] or 0:.2f}  wait {v['wait_mem_frac'] or 0:.2f}\")"
