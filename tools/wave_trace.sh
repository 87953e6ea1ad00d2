#!/bin/bash
# rocprofv3 kernel traces of tools/wave_probe's variants, one trace per
# variant, with every launch waited for (WP_SYNC=1): each dispatch runs on an
# idle GPU, so the trace's begin->end is the kernel's own duration,
# comparable across the empty kernel of the same grid, the descriptor load,
# phase 1 only and the dispatched kernel.
#   usage: tools/wave_trace.sh OUTDIR SIZE N [variants]
out=$1; size=${2:-1500}; n=${3:-4096}; vars=${4:-empty desc p1nl2 nl2 full g16 g4}
mkdir -p "$out"
export TMPDIR=/tmp
for v in $vars; do
  WP_SYNC=1 WP_ONLY=$v timeout -s KILL 120 \
    rocprofv3 --kernel-trace --stats -T --output-format csv -d "$out/$v" -o run -- \
    ./tools/wave_probe "$size" "$n" > "$out/$v.log" 2>&1 || exit $?
done
