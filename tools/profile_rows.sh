#!/bin/bash
# rocprofv3 kernel trace + stats of the f-row benches.
#   usage: tools/profile_rows.sh OUTDIR
out=$1
mkdir -p "$out"
export TMPDIR=/tmp
for c in f1 f3 f4; do
  timeout -s KILL 120 rocprofv3 --kernel-trace --stats -T --output-format csv -d "$out/$c" -o run -- \
      python3 bench.py --config $c --cpu-baseline off > "$out/$c.log" 2>&1 || exit $?
done
