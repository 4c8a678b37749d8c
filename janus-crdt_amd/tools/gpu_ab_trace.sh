#!/bin/bash
# Traced A/B (JANUS_TRACE_APPLY + JANUS_TRACE_MERGE) of the OR-Set apply loop: gpu_ab_trace.sh <out> <ENV_A> <ENV_B>
set -o pipefail
OUT=$1; A=$2; B=$3
mkdir -p "$OUT"
L="janus-crdt_amd/build/bench_orset --sets 2000 --msgs 200000 --waves 3 --cpu-msgs 0 --device 0 --direct"
for v in A B A B; do
  if [ $v = A ]; then E=$A; else E=$B; fi
  env $E JANUS_TRACE_APPLY=1 JANUS_TRACE_MERGE=1 timeout -k 10 120 $L > "$OUT/$v.json" 2> "$OUT/$v.err" || exit 1
  echo "== $v $E"; grep -E "apply tail|apply device|commit_tables|orset_node_check" "$OUT/$v.err" | tail -n 8
done
