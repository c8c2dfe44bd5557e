#!/bin/bash
# GPU-box run of chosen steps, each under its own time limit; a step that times out, aborts or segfaults ends
# the script.  Usage: bash tools/gpu_run.sh TAG STEP...   STEP = tests:<pytest args> | smoke | bench:<args> |
# prof:<bench args>
TAG=$1
shift
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # step NAME SECONDS CMD...
  local name=$1 secs=$2
  shift 2
  timeout -k 10 "$secs" "$@" > gpurun_out/${name}_$TAG.log 2>&1
  local rc=$?
  echo "$name EXIT $rc" >> gpurun_out/${name}_$TAG.log
  tail -n 4 gpurun_out/${name}_$TAG.log
  case $rc in
    124 | 134 | 137 | 139) echo "stopping after $name (exit $rc)"; exit $rc ;;
  esac
}
for s in "$@"; do
  case $s in
    tests:*) step test 1100 python -u -m pytest ${s#tests:} -s -v -rf --timeout 120 --timeout-method thread ;;
    smoke) step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench:*) step bench 600 python bench.py ${s#bench:} ;;
    # the trace database stays on the box (/tmp): only its summary comes back under gpurun_out/ (<= 64 MiB)
    prof:*) step prof 600 rocprofv3 --kernel-trace --stats -d /tmp/prof_$TAG -o run -- python bench.py ${s#prof:} &&
            python tools/rocprof_summary.py /tmp/prof_$TAG > gpurun_out/prof_summary_$TAG.md 2>&1 ;;
  esac
done
