#!/bin/bash
# PMC passes over the conv_tap kernels of tools/tap_bench.py (TAP_SHAPE selects shapes).
# usage: TAP_SHAPE=0 bash tools/tap_pmc.sh TAG
TAG=${1:-tappmc}
export TMPDIR=/tmp
mkdir -p gpurun_out
for spec in "sq:SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_INSTS_SALU" \
            "sq2:SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_MISC" \
            "tcc:TCC_HIT_sum TCC_MISS_sum"; do
  name=${spec%%:*}
  ctrs=${spec#*:}
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $ctrs --kernel-include-regex "conv_tap" -d gpurun_out/${TAG}_$name -o run -- python tools/tap_bench.py 3 > gpurun_out/${TAG}_$name.log 2>&1
  rc=$?
  echo "$name EXIT $rc"
  case $rc in 0) ;; *) exit $rc ;; esac
done
