set -o pipefail
mkdir -p gpurun_out/r2p
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_mlkem.py tests/test_gpu_edges.py tests/test_gpu_handshake.py tests/test_gpu_ordering.py tests/test_gpu_wire.py tests/test_gpu_hqc.py tests/test_gpu_frodo.py tests/test_abi.py > gpurun_out/r2p/t.log 2>&1 &&
timeout -k 10 200 python3 tools/single_shot_breakdown.py > gpurun_out/r2p/breakdown.json 2> gpurun_out/r2p/ss.err &&
QRKEM_LIBRARY=quantum-resistant-p2p_amd/qrkem/variants/libqrkem_sstrace.so timeout -k 10 200 python3 tools/single_shot_trace.py > gpurun_out/r2p/trace.json 2>> gpurun_out/r2p/ss.err
