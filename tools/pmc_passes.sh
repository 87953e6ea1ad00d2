#!/bin/bash
# PMC passes over one command (each pass a separate rocprofv3 run with
# --kernel-trace only, as MI355X_MICROARCH.md prescribes).  usage: pmc_passes.sh OUTDIR CMD...
out=$1; shift
mkdir -p "$out"
passes=(
  "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_INSTS_SMEM"
  "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA"
  "GRBM_GUI_ACTIVE SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"
  "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum"
  "TCC_HIT_sum TCC_MISS_sum"
  "FETCH_SIZE"
  "WRITE_SIZE"
)
i=0
for p in "${passes[@]}"; do
  rocprofv3 --pmc $p --kernel-trace -T --output-format csv -d "$out/pass$i" -o p -- "$@" > "$out/pass$i.log" 2>&1 || exit $?
  i=$((i+1))
done
