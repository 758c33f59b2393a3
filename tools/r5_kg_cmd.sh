# round 5: single-shot KeyGen pipeline check (tests + latency breakdown)
set -o pipefail
cd /root/repo && mkdir -p gpurun_out/r5/kg
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_mlkem.py tests/test_gpu_ordering.py > gpurun_out/r5/kg/tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/r5/kg/tests.log; exit 1; }
tail -3 gpurun_out/r5/kg/tests.log
for a in ML-KEM-768 ML-KEM-512 ML-KEM-1024; do
  timeout -k 10 120 python -u tools/single_shot_breakdown.py $a >> gpurun_out/r5/kg/breakdown.jsonl || exit $?
done
cat gpurun_out/r5/kg/breakdown.jsonl
