set -o pipefail
mkdir -p gpurun_out/r2g
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_mlkem.py tests/test_gpu_edges.py > gpurun_out/r2g/t.log 2>&1 &&
QRKEM_LIBRARY=quantum-resistant-p2p_amd/qrkem/variants/libqrkem_noslp.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_mlkem.py > gpurun_out/r2g/t_noslp.log 2>&1 &&
timeout -k 10 900 bash tools/ab.sh 3 default cmpcanon noslp -- --steps 10 --warmup 3 --streams 1 > gpurun_out/r2g/ab.jsonl 2> gpurun_out/r2g/ab.err
