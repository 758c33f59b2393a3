# HQC duplicate removal by readlane + ballot duplicate test (default) vs VGPR accumulators (variants/vreg):
# HQC GPU tests (crafted collisions vs the spec loop included) then A/B at 2^16.
set -o pipefail
O=gpurun_out/vreg
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_hqc.py tests/test_gpu_handshake.py > $O/t.log 2>&1 &&
timeout -k 10 300 bash tools/ab.sh 2 default vreg -- --alg HQC-128 > $O/ab_hqc128.jsonl 2> $O/ab.err &&
timeout -k 10 300 bash tools/ab.sh 1 default vreg -- --alg HQC-256 > $O/ab_hqc256.jsonl 2>> $O/ab.err
