#!/bin/bash
# per-variant PMC: SQ instruction mix of the wave probe's kernels
export TMPDIR=/tmp WP_ROUNDS=1
for v in ${WP_VARIANTS:-phase1 full g64}; do  # WP_ONLY matches substrings: name variants apart
  WP_ONLY=$v timeout -k 10 60 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_INSTS_SMEM --kernel-trace -T --output-format csv -d gpurun_out/pmcv/$v -o p -- ./tools/wave_probe 1500 4096 > gpurun_out/pmcv_$v.log 2>&1 || exit $?
  WP_ONLY=$v timeout -k 10 60 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS --kernel-trace -T --output-format csv -d gpurun_out/pmcv/${v}_b -o p -- ./tools/wave_probe 1500 4096 > gpurun_out/pmcv_${v}_b.log 2>&1 || exit $?
done
