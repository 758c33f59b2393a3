set -o pipefail
mkdir -p gpurun_out/r2j
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_mlkem.py tests/test_gpu_edges.py tests/test_gpu_handshake.py tests/test_gpu_ordering.py > gpurun_out/r2j/t.log 2>&1 &&
timeout -k 10 300 python3 tools/single_shot_latency.py > gpurun_out/r2j/single_shot.json && timeout -k 10 200 python3 tools/single_shot_breakdown.py > gpurun_out/r2j/breakdown.json 2> gpurun_out/r2j/ss.err &&
timeout -k 10 200 python3 bench.py --steps 10 --warmup 3 --no-cpu > gpurun_out/r2j/bench.json 2> gpurun_out/r2j/bench.err
