set -o pipefail
mkdir -p gpurun_out/ss2
g++ -O2 -Iinclude tools/oqs_latency.cpp -Lquantum-resistant-p2p_amd/qrkem -lqrkem -Wl,-rpath,$PWD/quantum-resistant-p2p_amd/qrkem -o /tmp/oqs_latency &&
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_mlkem.py tests/test_gpu_edges.py tests/test_gpu_handshake.py -k 'single_shot or edges or handshake or roundtrip' > gpurun_out/ss2/t.log 2>&1 &&
for a in HQC-128 HQC-192 HQC-256 FrodoKEM-640-AES FrodoKEM-640-SHAKE FrodoKEM-976-AES; do timeout -k 10 120 /tmp/oqs_latency $a 60 >> gpurun_out/ss2/c_api.json || exit 1; done &&
timeout -k 10 60 /tmp/oqs_latency ML-KEM-768 > gpurun_out/ss2/c_api_mlkem.json &&
timeout -k 10 60 /tmp/oqs_latency ML-KEM-512 >> gpurun_out/ss2/c_api_mlkem.json &&
timeout -k 10 60 /tmp/oqs_latency ML-KEM-1024 >> gpurun_out/ss2/c_api_mlkem.json &&
timeout -k 10 200 python3 tools/single_shot_breakdown.py > gpurun_out/ss2/breakdown.json 2> gpurun_out/ss2/ss.err &&
QRKEM_LIBRARY=quantum-resistant-p2p_amd/qrkem/variants/libqrkem_sstrace.so timeout -k 10 200 python3 tools/single_shot_trace.py > gpurun_out/ss2/trace.json 2>> gpurun_out/ss2/ss.err
