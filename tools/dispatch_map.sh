#!/bin/bash
# The dispatcher against every kernel it could pick (a measurement tool):
# for each batch size n, tools/size_sweep.py over frame sizes and mixes with
# the automatic choice (with and without the size hint) and each kernel
# forced (MTCP_GPU_SCHED), one process per n.  Output: gpurun_out/dispatch_map.jsonl; summary:
# python3 tools/dispatch_map.py gpurun_out/dispatch_map.jsonl
set -o pipefail
SIZES="64 128 256 512 768 1024 1500 2048 4096 9000 bimodal imix"
OUT=${OUT:-gpurun_out/dispatch_map.jsonl}
# every kernel choice of one batch size in one process, interleaved on the
# same buffers (tools/size_sweep.py --scheds)
for n in ${NS:-4096 16384 32768 65536 131072 262144 1048576}; do
  timeout -k 10 300 python -u tools/size_sweep.py --n $n --no-ceiling \
      --scheds ${SCHEDS:-auto,auto_hint,wave,row,quad,oct,span,big} $SIZES >> $OUT 2>/dev/null || exit 1
  echo "n=$n done"
done
