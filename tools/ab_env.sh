#!/bin/bash
# A/B of an environment switch on one box: the captured B=64 training step (tools/prof_step.py, K graph
# replays) with VAR=value for each value in turn, ROUNDS times interleaved.
# usage: [PREC=bf16] bash tools/ab_env.sh K ROUNDS VAR v1 v2 ...
export VITCNN_LIB=${VITCNN_LIB:-$(pwd)/vit-cnn_amd/vitcnn_amd/libvitcnn_probe.so}  # measurement knobs: the probe library
K=$1; ROUNDS=$2; VAR=$3; shift 3
for r in $(seq 1 $ROUNDS); do
  for v in "$@"; do
    out=$(env "$VAR=$v" timeout -k 10 120 python tools/prof_step.py $K ${PREC:-fp32} 2>&1 | grep "ms/step")
    rc=$?
    echo "round $r $VAR=$v: $out"
    case $rc in 0|1) ;; *) exit $rc ;; esac
  done
done
