# round 5, mid-size batches, final form: rho read from the keys with the context's parity fix-up
# counters at chunks <= 2^15 (no k_rho_copy).  ML-KEM parity tests, then same-box interleaved A/B
# against the round-5 docs head (abtrees/r5head).
set -o pipefail
cd /root/repo && source tools/gpu.sh
out r5/mid3
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_mlkem.py \
  tests/test_gpu_schedule.py tests/test_gpu_ordering.py > $O/tests_mlkem_mid3.log 2>&1 || { tail -30 $O/tests_mlkem_mid3.log; exit 1; }
tail -2 $O/tests_mlkem_mid3.log
out r5/mid3/ab14 && abx 4 new=default old=tree:abtrees/r5head -- --log2-batch 14 --steps 60 --warmup 10 --no-profile || exit 1
out r5/mid3/ab15 && abx 4 new=default old=tree:abtrees/r5head -- --log2-batch 15 --steps 40 --warmup 5 --no-profile || exit 1
out r5/mid3/ab16 && abx 2 new=default old=tree:abtrees/r5head -- --log2-batch 16 --steps 30 --warmup 5 --no-profile || exit 1
echo mid3_done
