#!/bin/bash
# A/B of environment switches on the FusAtNet B=64 training step (tools/fusat_step.py, one hipGraph), ROUNDS
# times interleaved; each SPEC is VAR=value[,VAR=value...] (or "base").  usage: bash tools/ab_fusat.sh STEPS ROUNDS SPEC...
export VITCNN_LIB=${VITCNN_LIB:-$(pwd)/vit-cnn_amd/vitcnn_amd/libvitcnn_probe.so}
STEPS=$1; ROUNDS=$2; shift 2
for r in $(seq 1 $ROUNDS); do
  for spec in "$@"; do
    if [ "$spec" = base ]; then set_env=(); else IFS=, read -r -a set_env <<< "$spec"; fi
    out=$(env "${set_env[@]}" timeout -k 10 300 python tools/fusat_step.py $STEPS 2>&1 | tail -1)
    rc=$?
    echo "round $r $spec: $(echo "$out" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], "ms/step, mfma_frac", d["mfma_frac"])' 2>&1 | tail -1)"
    case $rc in 0|1) ;; *) exit $rc ;; esac
  done
done
