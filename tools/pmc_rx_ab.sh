#!/bin/bash
# Instruction mix per wave of rx_kernel builds A and B on C2 (one rx_variants
# round, variant 0 = the dispatched kernel, plus its ablations), each counter
# set its own rocprofv3 pass.  usage: tools/pmc_rx_ab.sh OUTDIR VARIANTS_A VARIANTS_B
out=$1; a=$2; b=$3
export TMPDIR=/tmp
mkdir -p $out
for tag in a b; do
  exe=$a; [ $tag = b ] && exe=$b
  timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_INSTS_SMEM --kernel-trace -T --output-format csv -d $out/$tag -o p -- $exe c2 1 single > $out/$tag.log 2>&1 || exit $?
done
