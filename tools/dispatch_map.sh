#!/bin/bash
# The dispatcher against every kernel it could pick (a measurement tool):
# for each batch size n, tools/size_sweep.py over frame sizes and mixes with
# the automatic choice and each kernel forced (MTCP_GPU_SCHED), one process
# per (n, kernel).  Output: gpurun_out/dispatch_map.jsonl; summary:
# python3 tools/dispatch_map.py gpurun_out/dispatch_map.jsonl
set -o pipefail
SIZES="64 128 256 512 768 1024 1500 2048 4096 9000 bimodal imix"
for n in ${NS:-4096 16384 32768 65536 131072 262144 1048576}; do
  for s in ${SCHEDS:-auto wave row quad oct span big}; do
    if [ $s = auto ]; then unset MTCP_GPU_SCHED; else export MTCP_GPU_SCHED=$s; fi
    timeout -k 10 150 python -u tools/size_sweep.py --n $n --no-ceiling $SIZES >> gpurun_out/dispatch_map.jsonl 2>/dev/null || exit 1
  done
  echo "n=$n done"
done
