set -o pipefail
timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_fusatnet.py tests/test_conv_tap_gpu.py tests/test_bf16_gpu.py -rA > gpurun_out/fab_tests.log 2>&1; echo "tests rc=$?"; grep -E "argmax agreement|passed|failed" gpurun_out/fab_tests.log | tail -5
for r in 1 2; do for v in 26 22; do
  echo "SCRATCH=$v"; VITCNN_FUSAT_SCRATCH_LOG2=$v timeout -k 10 200 python tools/fusat_step.py 10 || exit $?
done; done
