#!/bin/bash
# PMC passes (one rocprofv3 --pmc run each, within the per-block counter limits) over 3 eager
# training steps of the B=64 ViT-CNN step (tools/run_steps.py), then per-kernel summaries:
#   sq   : VALU / SALU / LDS instruction counts, VALU-active and wave cycles, MFMA busy cycles, and
#          GRBM_GUI_ACTIVE (the denominator of the MFMA-busy and VALU-issue fractions)
#   fetch: FETCH_SIZE (HBM reads, KB)      write: WRITE_SIZE (HBM writes, KB)
# Usage: bash tools/pmc_step.sh TAG [fp32|bf16]
TAG=${1:-pmc}
PREC=${2:-fp32}
export TMPDIR=/tmp
mkdir -p gpurun_out
for spec in "sq:SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_INSTS_SALU GRBM_GUI_ACTIVE" "fetch:FETCH_SIZE" "write:WRITE_SIZE"; do
  name=${spec%%:*}
  ctrs=${spec#*:}
  timeout -s KILL 240 rocprofv3 --kernel-trace --pmc $ctrs -d gpurun_out/${TAG}_$name -o run -- python tools/run_steps.py 3 $PREC > gpurun_out/${TAG}_$name.log 2>&1
  rc=$?
  echo "$name EXIT $rc"
  case $rc in 0) ;; *) exit $rc ;; esac
done
python tools/pmc_summary.py gpurun_out/${TAG}_sq gpurun_out/${TAG}_fetch gpurun_out/${TAG}_write > gpurun_out/${TAG}_summary.txt 2>&1
