#!/bin/bash
# Dev (GPU box): SQ counters per dispatch for the json leg's kernels, one pass per counter set.
set -e
cd /tmp && export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS -d $O/pmc_json1 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --workload json --steps 4 --warmup 1 --no-cpu-baseline > $O/pmc_json1.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_INSTS_BRANCH SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_INSTS_SMEM -d $O/pmc_json2 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --workload json --steps 4 --warmup 1 --no-cpu-baseline > $O/pmc_json2.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum -d $O/pmc_json3 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --workload json --steps 4 --warmup 1 --no-cpu-baseline > $O/pmc_json3.log 2>&1
