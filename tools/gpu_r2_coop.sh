# Wave-cooperative sponges for small FrodoKEM / HQC batches: GPU tests (ragged small sizes hit the
# coop kernels, 2^16 full sizes the lane kernels), then C-API single-shot latency per algorithm.
set -o pipefail
O=gpurun_out/coop
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_frodo.py tests/test_gpu_hqc.py tests/test_gpu_handshake.py tests/test_gpu_fullsize.py > $O/t.log 2>&1 &&
g++ -O2 -Iinclude tools/oqs_latency.cpp -Lquantum-resistant-p2p_amd/qrkem -lqrkem -Wl,-rpath,$PWD/quantum-resistant-p2p_amd/qrkem -o /tmp/oqs_latency &&
rm -f $O/c_api.json &&
for a in HQC-128 HQC-192 HQC-256 FrodoKEM-640-AES FrodoKEM-640-SHAKE FrodoKEM-976-AES FrodoKEM-976-SHAKE FrodoKEM-1344-AES FrodoKEM-1344-SHAKE; do timeout -k 10 120 /tmp/oqs_latency $a 60 >> $O/c_api.json || exit 1; done
