#!/bin/bash
# Dev (GPU box): C5 apply-loop wall time, whole process pinned to either NUMA node vs unpinned, alternated.
O=$GRAFT_REPO_ROOT/gpurun_out/probe3
mkdir -p $O
python3 -c "import torch;p=torch.cuda.get_device_properties(0);print(p.pci_domain_id,p.pci_bus_id,p.pci_device_id)" > $O/gpu.txt 2>&1
for d in /sys/bus/pci/devices/*; do [ -f $d/class ] && grep -q 0x038 $d/class 2>/dev/null && echo "$d $(cat $d/numa_node)"; done >> $O/gpu.txt 2>&1
B=./janus-crdt_amd/build/bench_apply
run() { local tag=$1; shift; timeout -k 10 200 "$@" --waves 3 --cpu-msgs 0 > $O/$tag.json 2> $O/$tag.err || exit 1; }
for r in 1 2 3; do
  run base$r $B
  run node0_$r taskset -c 0-63,128-191 $B
  run node1_$r taskset -c 64-127,192-255 $B
done
echo probe3-done
