set -o pipefail
timeout -k 10 400 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_fusatnet.py tests/test_conv_tap_gpu.py -rA > gpurun_out/fab_tests.log 2>&1; echo "tests rc=$?"; grep -E "passed|failed" gpurun_out/fab_tests.log | tail -5
timeout -k 10 300 python -u tools/bf16_sites.py
