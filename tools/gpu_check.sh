#!/bin/bash
# GPU-box check: parity tests, smoke, bench, kernel-trace profile. Usage: bash tools/gpu_check.sh TAG
# Each GPU step has its own time limit; a step that times out, aborts or segfaults ends the script
# (ordinary test failures, exit 1, do not).
TAG=${1:-run}
mkdir -p gpurun_out
export TMPDIR=/tmp

step() {  # step NAME SECONDS CMD...
  local name=$1 secs=$2
  shift 2
  timeout -k 10 "$secs" "$@" > gpurun_out/${name}_$TAG.log 2>&1
  local rc=$?
  echo "$name EXIT $rc" >> gpurun_out/${name}_$TAG.log
  tail -n 3 gpurun_out/${name}_$TAG.log
  case $rc in
    124 | 134 | 137 | 139) echo "stopping after $name (exit $rc)"; exit $rc ;;
  esac
}

step test 600 python -u -m pytest tests/ -m gpu -q -rf --timeout 120 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench 600 python bench.py --steps 100 --warmup 10 ${BENCH_ARGS}
step prof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline
python tools/rocprof_summary.py gpurun_out/prof_$TAG > gpurun_out/prof_summary_$TAG.md 2>&1 || true
