set -o pipefail
mkdir -p gpurun_out/r05/cb8
export TMPDIR=/tmp
L="janus-crdt_amd/build/bench_orset --sets 2000 --msgs 200000 --waves 3 --cpu-msgs 0 --device 0 --direct"
for i in 1 2 3; do timeout -k 10 120 $L > gpurun_out/r05/cb8/run$i.json 2>gpurun_out/r05/cb8/run$i.err || exit 1; python3 -c "import json;print(json.loads(open('gpurun_out/r05/cb8/run$i.json').read().strip().splitlines()[-1])['ms_per_wave'])"; done
JANUS_TRACE_APPLY=1 JANUS_TRACE_MERGE=1 timeout -k 10 120 $L > /dev/null 2> gpurun_out/r05/cb8/trace.err || exit 1
grep -E "apply device|commit_tables" gpurun_out/r05/cb8/trace.err
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r05/cb8/kt -o run --output-format csv -- $L > gpurun_out/r05/cb8/kt.out 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_orset_wire_gpu.py tests/test_node_gpu.py -m gpu > gpurun_out/r05/cb8/pytest.log 2>&1; rc=$?; tail -3 gpurun_out/r05/cb8/pytest.log; exit $rc
