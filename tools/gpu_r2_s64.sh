# A/B: Keccak rotations on 64-bit shifts (QRK_KECCAK_SHIFT64=1, variants/libqrkem_s64.so) vs
# the default alignbit build, interleaved in one call, then the GPU suite on the variant.
set -o pipefail
O=gpurun_out/s64
mkdir -p $O
timeout -k 10 400 bash tools/ab.sh 2 default s64 -- > $O/ab_mlkem768.jsonl 2> $O/ab.err &&
timeout -k 10 300 bash tools/ab.sh 2 default s64 -- --alg FrodoKEM-640-SHAKE > $O/ab_frodo640.jsonl 2>> $O/ab.err &&
timeout -k 10 300 bash tools/ab.sh 2 default s64 -- --alg HQC-128 > $O/ab_hqc128.jsonl 2>> $O/ab.err &&
QRKEM_LIBRARY=$PWD/quantum-resistant-p2p_amd/qrkem/variants/libqrkem_s64.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_mlkem.py tests/test_gpu_frodo.py tests/test_gpu_hqc.py tests/test_gpu_handshake.py > $O/t.log 2>&1
