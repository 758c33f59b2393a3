# HQC decode dedupe spread over all waves (QRK_HQC_DEDUPE_WG=1) vs wave 0 alone
# (variants/libqrkem_dwg0.so): HQC GPU tests, then A/B.
set -o pipefail
O=gpurun_out/dwg
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_hqc.py tests/test_gpu_handshake.py > $O/t.log 2>&1 &&
timeout -k 10 400 bash tools/ab.sh 2 default dwg0 -- --alg HQC-192 > $O/ab_hqc192.jsonl 2> $O/ab.err &&
timeout -k 10 400 bash tools/ab.sh 2 default dwg0 -- --alg HQC-256 > $O/ab_hqc256.jsonl 2>> $O/ab.err &&
timeout -k 10 300 bash tools/ab.sh 1 default dwg0 -- --alg HQC-128 > $O/ab_hqc128.jsonl 2>> $O/ab.err
