set -o pipefail
mkdir -p gpurun_out/r2z
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_hqc.py tests/test_gpu_handshake.py > gpurun_out/r2z/t.log 2>&1 &&
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_fullsize.py -k "hqc or HQC" >> gpurun_out/r2z/t.log 2>&1 &&
QRKEM_LIBRARY=quantum-resistant-p2p_amd/qrkem/variants/libqrkem_hqctrace.so timeout -k 10 200 python3 tools/hqc_trace.py > gpurun_out/r2z/hqc_trace.json 2> gpurun_out/r2z/hqc.err &&
timeout -k 10 300 python3 bench.py --alg HQC-128 --no-cpu > gpurun_out/r2z/hqc128.json 2> gpurun_out/r2z/b.err &&
timeout -k 10 300 python3 bench.py --alg HQC-256 --no-cpu > gpurun_out/r2z/hqc256.json 2>> gpurun_out/r2z/b.err
