#!/bin/bash
# FETCH_SIZE / WRITE_SIZE passes (each its own run) over one bench config.
#   usage: tools/pmc_row.sh CONFIG OUTDIR
cfg=$1; out=$2
mkdir -p "$out"
export TMPDIR=/tmp
b="python3 bench.py --config $cfg --steps 20 --warmup 2 --cpu-baseline off --pcie off"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -T --output-format csv -d "$out/fetch" -o run -- $b > "$out/fetch.log" 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace -T --output-format csv -d "$out/write" -o run -- $b > "$out/write.log" 2>&1 || exit $?
