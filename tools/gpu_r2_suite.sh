set -o pipefail
mkdir -p gpurun_out/suite
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/suite/t.log 2>&1 &&
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/suite/smoke.log 2>&1 &&
timeout -k 10 300 python3 bench.py --alg HQC-128 > gpurun_out/suite/hqc128.json 2> gpurun_out/suite/b.err &&
timeout -k 10 300 python3 bench.py --alg HQC-192 > gpurun_out/suite/hqc192.json 2>> gpurun_out/suite/b.err &&
timeout -k 10 300 python3 bench.py --alg HQC-256 > gpurun_out/suite/hqc256.json 2>> gpurun_out/suite/b.err &&
timeout -k 10 300 python3 bench.py --alg HQC-128 --mode decaps-tampered > gpurun_out/suite/hqc128_tampered.json 2>> gpurun_out/suite/b.err &&
timeout -k 10 300 python3 bench.py --alg HQC-128 --mode handshake > gpurun_out/suite/handshake_hqc128.json 2>> gpurun_out/suite/b.err
