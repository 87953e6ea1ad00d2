#!/bin/bash
# FETCH_SIZE per rx_variants kernel (C5)
cd /root/repo
export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --kernel-trace -T --output-format csv -d gpurun_out/pmcv -o run -- ./tools/rx_variants c5 1 > gpurun_out/pmcv.log 2>&1
