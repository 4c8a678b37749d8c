#!/bin/bash
# Counters of the OR-Set wire path (the apply loop's per-chunk parse + table kernels and its commit tail) and
# the JSON pass A, each counter group in a pass of its own (rocprofv3 does not split passes), plus a kernel +
# copy timeline of the page-locked OR-Set wave.  Usage: gpu_pmc_orset.sh <outdir>
set -o pipefail
OUT=${1:-gpurun_out/pmc_orset}
export TMPDIR=/tmp
mkdir -p "$OUT"
ORSET="janus-crdt_amd/build/bench_orset --sets 2000 --msgs 200000 --waves 2 --cpu-msgs 0 --device 0 --direct"
JSON="python3 bench.py --steps 4 --warmup 1 --no-cpu-baseline --workload json"
SQ1=SQ_INSTS_VALU,SQ_INSTS_SALU,SQ_INSTS_LDS,SQ_INSTS_VMEM,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_WAVE_CYCLES,SQ_BUSY_CYCLES
SQ2=SQ_ACTIVE_INST_ANY,SQ_INSTS_SMEM,SQ_WAIT_INST_LDS,SQ_LDS_BANK_CONFLICT,SQ_LDS_IDX_ACTIVE
TCC=TCC_ATOMIC_sum,TCC_HIT_sum,TCC_MISS_sum,TCC_EA0_RDREQ_sum
pass() {  # pass <name> <counters> <command...>
    local name=$1 ctr=$2
    shift 2
    timeout -s KILL 150 rocprofv3 --pmc "$ctr" -d "$OUT/$name" -o run --output-format csv -- "$@" > "$OUT/$name.out" 2>&1 || exit 1
    echo "pass $name done"
}
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace -d "$OUT/timeline" -o run --output-format csv -- $ORSET > "$OUT/timeline.out" 2>&1 || exit 1
echo "timeline done"
pass orset_fetch FETCH_SIZE $ORSET
pass orset_write WRITE_SIZE $ORSET
pass orset_sq1 $SQ1 $ORSET
pass orset_sq2 $SQ2 $ORSET
pass orset_tcc $TCC $ORSET
pass json_sq1 $SQ1 $JSON
pass json_sq2 $SQ2 $JSON
echo pmc-orset-done
