a=$1; b=$2; n=${3:-4}
for i in $(seq 1 $n); do
  for d in $a $b; do
    (cd $d && timeout -k 10 120 python bench.py --config c3 --record compact --cpu-baseline off --pcie off --small-batch off --ceiling off) | grep '^{' | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); print('$d', d['roofline']['avg_launch_ms']*1e3, d['roofline']['frac'])" || exit 1
  done
done
