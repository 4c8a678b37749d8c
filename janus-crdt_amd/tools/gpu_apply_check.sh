#!/bin/bash
# GPU suite, then the three apply-loop benches (C5 twice, OR-Set, C1), each step under its own limit.
S=janus-crdt_amd/tools/gpu_steps.sh
bash $S pytest_gpu.log 600 python -u -m pytest tests/test_abi.py tests/test_node_gpu.py tests/test_apply_loop_gpu.py -x -q --timeout 120 --timeout-method thread && \
bash $S ap_c5a.log 120 janus-crdt_amd/build/bench_apply --accounts 1000000 --ops 1000000 --waves 3 --cpu-msgs 0 --device 0 && \
bash $S ap_orset.log 120 janus-crdt_amd/build/bench_orset --sets 2000 --msgs 200000 --waves 3 --cpu-msgs 0 --device 0 && \

bash $S ap_c5b.log 120 janus-crdt_amd/build/bench_apply --accounts 1000000 --ops 1000000 --waves 3 --cpu-msgs 0 --device 0
