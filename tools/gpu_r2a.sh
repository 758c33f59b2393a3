set -o pipefail
mkdir -p gpurun_out/r2a
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_ordering.py tests/test_gpu_configs2.py tests/test_gpu_multirank.py > gpurun_out/r2a/new_tests.log 2>&1 &&
timeout -k 10 300 python3 bench.py --global-log2-batch 24 --steps 3 --warmup 1 > gpurun_out/r2a/bench_cfg2.json 2> gpurun_out/r2a/bench_cfg2.err &&
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/r2a/gpu_all.log 2>&1
