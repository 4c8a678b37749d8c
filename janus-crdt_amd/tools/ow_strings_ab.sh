#!/bin/bash
# A/B of OR-Set wave-table builds under kernel trace (round 6): each directory janus-crdt_amd/lib/<v>/ holds a
# libjanusgpu.so built with the change under test (bench_orset's RUNPATH yields to LD_LIBRARY_PATH); prints
# ms_per_wave and the per-wave time of k_ow_group / k_ow_strings / k_ow_rins (5 waves + 2 warm-ups = 7).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r06/owab
mkdir -p $OUT
for v in exp_base exp_nosame exp_base; do
  for r in 1 2; do
    d=$OUT/${v}_$r
    LD_LIBRARY_PATH=$PWD/janus-crdt_amd/lib/$v timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $d -o run --output-format csv -- janus-crdt_amd/build/bench_orset --sets 2000 --msgs 200000 --waves 5 --cpu-msgs 0 --device 0 --direct > $d.json 2> $d.err || exit 1
    python3 - $d <<'PY'
import csv,glob,sys,json
d=sys.argv[1]
f=glob.glob(d+'/**/*kernel_stats.csv',recursive=True)[0]
tot={r['Name'][:40]:(int(r['Calls']),float(r['TotalDurationNs'])) for r in csv.DictReader(open(f))}
ks={k:v for k,v in tot.items() if 'k_ow_strings' in k or 'k_ow_group' in k or 'k_ow_rins' in k}
j=json.loads(open(d+'.json').read().strip().splitlines()[-1])
print(d.split('/')[-1], j['ms_per_wave'], {k[22:36]:(c, round(t/1e3/7,1)) for k,(c,t) in ks.items()})
PY
  done
done
