#!/bin/bash
# FusAtNet B = 4 backward accuracy under the conv / scratch knobs (diagnostic; GPU box)
set -o pipefail
timeout -k 10 300 python -u -m pytest -q --timeout 150 --timeout-method thread tests/test_conv_tap_gpu.py > gpurun_out/tap_bisect.log 2>&1
echo "tap tests rc=$?"; tail -5 gpurun_out/tap_bisect.log
export VITCNN_LIB=${VITCNN_LIB:-$(pwd)/vit-cnn_amd/vitcnn_amd/libvitcnn_probe.so}  # measurement knobs: the probe library
for cfg in "VITCNN_FUSAT_IM2COL=1 VITCNN_FUSAT_SCRATCH_LOG2=26" "VITCNN_TAP_NOSPLIT=1 VITCNN_FUSAT_SCRATCH_LOG2=22" \
           "VITCNN_FUSAT_SCRATCH_LOG2=22" "VITCNN_FUSAT_SCRATCH_LOG2=23"; do
  echo "=== $cfg"
  env $cfg timeout -k 10 200 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_fusatnet.py -k "backward_b4" 2>&1 | tail -1
  rc=$?
  python -c "
import json,os
p='gpurun_out/fusat_grad_b4.json'
if os.path.exists(p):
    b=json.load(open(p)); print(len(b), [(k, round(e/n,6)) for k,e,e32,n in b[:3]]); os.remove(p)
"
  [ $rc -ge 124 ] && exit $rc
done
exit 0
