#!/bin/bash
# Dev sweep (GPU box): bench.py's device-resident json leg at each JANUS_JSON_GROUP, kernel stats per setting.
set -e
cd /tmp && export TMPDIR=/tmp
for G in ${JG_SWEEP:-1 4 8 16}; do
  JANUS_JSON_GROUP=$G timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/sweep_g$G -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --workload json --steps 10 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/sweep_g$G.log 2>&1
done
