# round-2 refresh: whole GPU suite, default bench, configs[2] bench, single-shot latency,
# ML-KEM-768 2^20 rocprof trace + FETCH/WRITE + SQ passes
set -o pipefail
mkdir -p gpurun_out/r2x
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/r2x/t.log 2>&1 &&
timeout -k 10 300 python3 bench.py > gpurun_out/r2x/bench.json 2> gpurun_out/r2x/bench.err &&
timeout -k 10 300 python3 bench.py --global-log2-batch 24 --steps 3 --warmup 1 > gpurun_out/r2x/bench_configs2.json 2> gpurun_out/r2x/bench_configs2.err &&
timeout -k 10 300 python3 tools/single_shot_latency.py > gpurun_out/r2x/single_shot.json 2> gpurun_out/r2x/ss.err &&
bash tools/profile.sh mlkem768_r2 > gpurun_out/r2x/prof.log 2>&1 &&
bash tools/pmc_sq.sh mlkem768_r2 > gpurun_out/r2x/sq.log 2>&1
