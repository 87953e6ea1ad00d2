#!/bin/bash
# Interleaved A/B of the small-batch kernels (tools/wave_probe, built in each
# tree): tools/ab_wave_probe.sh DIR_A DIR_B ROUNDS
a=${1:-abA}; b=${2:-.}; n=${3:-3}
for i in $(seq 1 $n); do for d in $a $b; do
  for spec in "1500 4096 8192 16384" "64 2048 4096 16384 65536" "9000 4096"; do
    (cd $d && timeout -k 10 60 ./tools/wave_probe $spec) | sed "s|^|{\"tree\":\"$d\"} |" || exit 1
  done
done; done
