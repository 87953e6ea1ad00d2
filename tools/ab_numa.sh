#!/bin/bash
# Interleaved A/B of bench.py's host binding (--numa on | off): the
# PCIe-inclusive leg and the CPU baseline, three rounds on one box.
#   /usr/local/graft/bin/gpurun -- 'bash tools/ab_numa.sh'
mkdir -p gpurun_out
python3 -c "
import json, os
from mtcp_amd import gpu
bdf, cpus = gpu.device_local_cpus(0)
print(json.dumps({'probe': 'host_topology', 'gpu_pci': bdf, 'local_cpus': sorted(cpus),
                  'allowed': len(os.sched_getaffinity(0))}))" > gpurun_out/ab_numa.jsonl || exit 1
for r in 1 2 3; do
  for m in on off; do
    timeout -k 10 150 python3 bench.py --numa $m --small-batch off > gpurun_out/ab_numa_$m.log 2>&1 || exit $?
    python3 -c "
import json, sys
l = [x for x in open('gpurun_out/ab_numa_$m.log') if x.startswith('{')][-1]
b = json.loads(l)
print(json.dumps({'round': $r, 'numa': '$m', 'value': b['value'], 'frac': b['roofline']['frac'],
                  'pcie_inclusive': b['pcie_inclusive']['value'], 'cpu_gbs': b['cpu_baseline']['value'],
                  'cpu_per_core_count': b['cpu_baseline']['per_core_count'], 'host_cpus': b['host_cpus']}))" >> gpurun_out/ab_numa.jsonl || exit 1
  done
done
cat gpurun_out/ab_numa.jsonl
