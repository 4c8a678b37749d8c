#!/bin/bash
# Dev (GPU box): C5 apply-loop host time vs NUMA placement and classify prefetch distance.
O=$GRAFT_REPO_ROOT/gpurun_out/probe2
mkdir -p $O
{ for f in /sys/class/drm/card*/device/numa_node; do echo "$f $(cat $f)"; done; cat /sys/fs/cgroup/cpuset.cpus.effective; } > $O/host.txt 2>&1
B=./janus-crdt_amd/build/bench_apply
run() { local tag=$1; shift; JANUS_TRACE_WAVE=1 timeout -k 10 200 "$@" --waves 3 --cpu-msgs 0 > $O/$tag.json 2> $O/$tag.trace || exit 1; }
run base $B
run node0 taskset -c 0-63,128-191 $B
run node1 taskset -c 64-127,192-255 $B
JANUS_PF=16 run pf16 $B
JANUS_PF=32 run pf32 $B
echo probe2-done
