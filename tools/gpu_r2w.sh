set -o pipefail
mkdir -p gpurun_out/r2w
g++ -O2 -Iinclude tools/oqs_latency.cpp -Lquantum-resistant-p2p_amd/qrkem -lqrkem -Wl,-rpath,$PWD/quantum-resistant-p2p_amd/qrkem -o /tmp/oqs_latency &&
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_mlkem.py tests/test_gpu_edges.py tests/test_gpu_handshake.py tests/test_gpu_ordering.py tests/test_abi.py > gpurun_out/r2w/t.log 2>&1 &&
timeout -k 10 60 /tmp/oqs_latency ML-KEM-768 > gpurun_out/r2w/c_api.json &&
timeout -k 10 60 /tmp/oqs_latency ML-KEM-512 >> gpurun_out/r2w/c_api.json &&
timeout -k 10 60 /tmp/oqs_latency ML-KEM-1024 >> gpurun_out/r2w/c_api.json &&
timeout -k 10 200 python3 tools/single_shot_breakdown.py > gpurun_out/r2w/breakdown.json 2> gpurun_out/r2w/ss.err && QRKEM_LIBRARY=quantum-resistant-p2p_amd/qrkem/variants/libqrkem_sstrace.so timeout -k 10 200 python3 tools/single_shot_trace.py > gpurun_out/r2w/trace.json 2>> gpurun_out/r2w/ss.err
