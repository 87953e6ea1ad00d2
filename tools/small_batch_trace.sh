#!/bin/bash
# rocprofv3 kernel traces of the small-batch kernels through the C-ABI.
#   usage: tools/small_batch_trace.sh OUTDIR [graph]
out=$1; mode=$2
mkdir -p "$out"
export TMPDIR=/tmp
for s in 1500 9000 64 bimodal; do
  timeout -s KILL 120 rocprofv3 --kernel-trace --stats -T --output-format csv -d "$out/$s" -o run -- \
      python3 tools/small_batch_trace.py $s 4096 200 $mode > "$out/$s.log" 2>&1 || exit $?
done
