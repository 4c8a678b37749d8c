#!/bin/bash
# Dev (GPU box): VALU / SALU instruction counts per dispatch of the json leg (one --pmc pass).
cd /tmp && export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/prof
mkdir -p $O
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAIT_INST_ANY -d $O/sq_json -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --workload json --steps 4 --warmup 1 --no-cpu-baseline > $O/sq_json.log 2>&1
