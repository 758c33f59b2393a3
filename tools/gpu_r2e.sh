set -o pipefail
mkdir -p gpurun_out/r2e
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_frodo.py tests/test_gpu_fullsize.py -k "Frodo or frodo" > gpurun_out/r2e/t.log 2>&1 &&
timeout -k 10 600 bash tools/ab.sh 2 default kgrows -- --mode handshake --alg FrodoKEM-976-SHAKE --steps 3 --warmup 1 > gpurun_out/r2e/ab976.jsonl 2> gpurun_out/r2e/ab976.err &&
timeout -k 10 600 bash tools/ab.sh 2 default kgrows -- --mode handshake --alg FrodoKEM-640-SHAKE --steps 3 --warmup 1 > gpurun_out/r2e/ab640.jsonl 2> gpurun_out/r2e/ab640.err
