#!/bin/bash
# rocprofv3 evidence for one bench config, each pass its own run:
#   1. --kernel-trace --stats (durations)
#   2. --pmc FETCH_SIZE          3. --pmc WRITE_SIZE
#   4. --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_64B_sum
# usage: tools/profile_config.sh CONFIG OUTDIR
#   CONFIG: c1 c2 c3 c5 (bench configs), c3_compact (c3 with 16 B records), f1, f3
cfg=$1; out=$2
mkdir -p "$out"
export TMPDIR=/tmp
case "$cfg" in
  *_compact) bargs="--config ${cfg%_compact} --record compact" ;;
  *)         bargs="--config $cfg" ;;
esac
sha256sum mtcp_amd/lib/libmtcp_gpu.so | cut -d' ' -f1 > "$out/lib.sha256"   # the build profiled
python3 -c "from mtcp_amd import _codeobj; print(_codeobj.rx_source_key())" > "$out/rx_source.key"
b="python3 bench.py $bargs --steps 200 --warmup 20 --cpu-baseline off --pcie off --small-batch off --ceiling off --c4-per-gpu off"
timeout -s KILL 150 rocprofv3 --kernel-trace --stats -T --output-format csv -d "$out/trace" -o run -- $b > "$out/trace.log" 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -T --output-format csv -d "$out/fetch" -o run -- $b > "$out/fetch.log" 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace -T --output-format csv -d "$out/write" -o run -- $b > "$out/write.log" 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_64B_sum --kernel-trace -T --output-format csv -d "$out/rdreq" -o run -- $b > "$out/rdreq.log" 2>&1 || exit $?
