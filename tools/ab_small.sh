#!/bin/bash
# A/B of two builds (each DIR a repo tree with its lib and tools/wave_probe
# built), runs interleaved on one box: bench.py's kernel time and small-batch
# line for each CONFIG, then the wave probe at 4 096 packets of each size.
#   tools/ab_small.sh DIR_A DIR_B ROUNDS CONFIG...
a=$1; b=$2; n=$3; shift 3
for i in $(seq 1 $n); do
  for cfg in "$@"; do
    for d in $a $b; do
      (cd $d && timeout -k 10 120 python bench.py --config $cfg --cpu-baseline off --pcie off) | grep '^{' | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); sb=d.get('small_batch',{})
print(json.dumps({'tree':'$d','config':'$cfg','round':$i,'kernel_us':round(d['roofline']['avg_launch_ms']*1e3,2),'frac':d['roofline']['frac'],'small_batch_us':sb.get('us_per_launch')}))" || exit 1
    done
  done
  for d in $a $b; do
    for size in 1500 64 9000; do
      (cd $d && timeout -k 10 60 ./tools/wave_probe $size 4096 16384) | sed "s|^|{\"tree\":\"$d\",\"size\":$size} |" || exit 1
    done
  done
done
