set -o pipefail
mkdir -p gpurun_out/t3
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/t3/t.log 2>&1 &&
timeout -k 10 300 python3 tools/small_crossover.py new > gpurun_out/t3/cross.json 2> gpurun_out/t3/err &&
timeout -k 10 300 python3 bench.py --steps 10 --warmup 3 --no-cpu > gpurun_out/t3/bench.json 2>> gpurun_out/t3/err
