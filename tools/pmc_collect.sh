#!/bin/bash
# PMC passes over a few eager training steps (separate passes: FETCH_SIZE and WRITE_SIZE do not fit
# one TCC pass on gfx950).  Usage: bash tools/pmc_collect.sh TAG
TAG=${1:-pmc}
export TMPDIR=/tmp
mkdir -p gpurun_out
for spec in "fetch:FETCH_SIZE" "write:WRITE_SIZE" "sq:SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS"; do
  name=${spec%%:*}
  ctrs=${spec#*:}
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $ctrs -d gpurun_out/${TAG}_$name -o run -- python tools/run_steps.py 3 > gpurun_out/${TAG}_$name.log 2>&1
  rc=$?
  echo "$name EXIT $rc"
  case $rc in 0) ;; *) exit $rc ;; esac
done
