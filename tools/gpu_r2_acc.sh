# A/B: SampleNTT acceptance as a shifted difference (QRK_XOF_ACC=1, default build) vs the
# v_cmp + v_cndmask compaction (variants/libqrkem_acc0.so); ML-KEM GPU tests on the default.
set -o pipefail
O=gpurun_out/acc
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_mlkem.py tests/test_gpu_edges.py > $O/t.log 2>&1 &&
timeout -k 10 600 bash tools/ab.sh 3 default acc0 -- > $O/ab_mlkem768.jsonl 2> $O/ab.err
