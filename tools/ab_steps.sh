#!/bin/bash
# A/B of library builds on one box: the captured B=64 training step (tools/prof_step.py, K graph
# replays) with VITCNN_LIB pointing at each build in turn, ROUNDS times interleaved.
# usage: bash tools/ab_steps.sh K ROUNDS lib1.so lib2.so ...   (a path "cur" = the in-tree build)
K=$1; ROUNDS=$2; shift 2
for r in $(seq 1 $ROUNDS); do
  for lib in "$@"; do
    if [ "$lib" = cur ]; then unset VITCNN_LIB; else export VITCNN_LIB=$lib; fi
    out=$(timeout -k 10 120 python tools/prof_step.py $K 2>&1 | grep "ms/step")
    rc=$?
    echo "round $r $lib: $out"
    case $rc in 0|1) ;; *) exit $rc ;; esac
  done
done
