#!/bin/bash
# A/B of two builds of the product on one box, runs interleaved:
#   tools/ab_bench.sh DIR_A DIR_B CONFIG ROUNDS    (each DIR a repo tree with its lib built)
a=$1; b=$2; cfg=$3; n=${4:-4}
for i in $(seq 1 $n); do
  for d in $a $b; do
    (cd $d && timeout -k 10 120 python bench.py --config $cfg --cpu-baseline off --pcie off) | grep '^{' | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); print('$d', d['roofline']['avg_launch_ms']*1e3, d['roofline']['frac'])" || exit 1
  done
done
