set -o pipefail
OUT=gpurun_out/mab; mkdir -p $OUT
for i in 1 2 3; do
  timeout -k 10 200 janus-crdt_amd/build/bench_submit --workload pnc --keys 1000000 --ops 1000000 --waves 3 --cpu-ops 20000 --device 0 > $OUT/p$i.json 2>/dev/null || exit 1
  MALLOC_MMAP_THRESHOLD_=33554432 MALLOC_TRIM_THRESHOLD_=17179869184 timeout -k 10 200 janus-crdt_amd/build/bench_submit --workload pnc --keys 1000000 --ops 1000000 --waves 3 --cpu-ops 20000 --device 0 > $OUT/m$i.json 2>/dev/null || exit 1
  python3 -c "
import json
for v in ('p','m'):
    d=json.loads(open('$OUT/'+v+'$i.json').read().strip().splitlines()[-1]); print(v, d['ms_per_wave'], d['parity_vs_oracle'])"
done
MALLOC_MMAP_THRESHOLD_=33554432 MALLOC_TRIM_THRESHOLD_=17179869184 JANUS_TRACE_SUBMIT=1 timeout -k 10 200 janus-crdt_amd/build/bench_submit --workload pnc --keys 1000000 --ops 1000000 --waves 3 --cpu-ops 20000 --device 0 > $OUT/tm.json 2> $OUT/tm.err
