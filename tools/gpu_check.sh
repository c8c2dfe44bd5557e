set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_model_gpu.py -q -rf > gpurun_out/t3.log 2>&1; echo "TEST EXIT $?" >> gpurun_out/t3.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke3.log 2>&1; echo "SMOKE EXIT $?" >> gpurun_out/smoke3.log
timeout -k 10 600 python bench.py --steps 50 --warmup 10 > gpurun_out/bench3.log 2>&1; echo "BENCH EXIT $?" >> gpurun_out/bench3.log
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof3 -o run -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/prof3.log 2>&1; echo "PROF EXIT $?" >> gpurun_out/prof3.log
tail -3 gpurun_out/t3.log gpurun_out/smoke3.log gpurun_out/bench3.log gpurun_out/prof3.log
