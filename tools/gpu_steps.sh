#!/bin/bash
# Run GPU steps in order, each under its own time limit: "bash tools/gpu_steps.sh TAG 'name:secs:cmd' ...".
# A step that times out, aborts or segfaults ends the script; ordinary failures (exit 1) do not.
TAG=$1
shift
mkdir -p gpurun_out
export TMPDIR=/tmp
for spec in "$@"; do
  name=${spec%%:*}
  rest=${spec#*:}
  secs=${rest%%:*}
  cmd=${rest#*:}
  timeout -k 10 "$secs" bash -c "$cmd" > gpurun_out/${name}_$TAG.log 2>&1
  rc=$?
  echo "$name EXIT $rc" | tee -a gpurun_out/${name}_$TAG.log
  case $rc in
    124 | 134 | 137 | 139) echo "stopping after $name (exit $rc)"; exit $rc ;;
  esac
done
