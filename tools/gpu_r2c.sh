set -o pipefail
mkdir -p gpurun_out/r2c
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_mlkem.py > gpurun_out/r2c/t.log 2>&1 &&
timeout -k 10 600 bash tools/ab.sh 3 default cmp -- --steps 10 --warmup 3 --streams 1 > gpurun_out/r2c/ab.jsonl 2> gpurun_out/r2c/ab.err
