#!/bin/bash
# PMC + kernel-trace of one GEMM shape under each kernel variant (tools/gemm_one.py).
# usage: bash tools/gemm_pmc.sh TAG "TA TB M N K" [flags...]
TAG=$1
SHAPE=$2
shift 2
export TMPDIR=/tmp
mkdir -p gpurun_out
for fl in "$@"; do
  timeout -k 10 120 python tools/gemm_one.py $SHAPE $fl 200 >> gpurun_out/${TAG}_time.log 2>&1 || exit $?
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_f${fl}_kt -o run -- python tools/gemm_one.py $SHAPE $fl 50 > /dev/null 2>&1 || exit $?
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE -d gpurun_out/${TAG}_f${fl}_sq -o run -- python tools/gemm_one.py $SHAPE $fl 50 > /dev/null 2>&1 || exit $?
  python tools/pmc_summary.py gpurun_out/${TAG}_f${fl}_sq --filter gemm >> gpurun_out/${TAG}_pmc.log 2>&1
  python tools/rocprof_summary.py gpurun_out/${TAG}_f${fl}_kt >> gpurun_out/${TAG}_kt.log 2>&1
  rm -rf gpurun_out/${TAG}_f${fl}_kt gpurun_out/${TAG}_f${fl}_sq
done
