# round 5, mid-size batches: rho read from the keys + parity fix-up counters (no k_rho_copy at chunks
# <= 2^16), G(m' || h) inside the decrypt role (no k_g_decaps at chunks <= 2^15).  ML-KEM parity
# tests, then same-box interleaved A/B against the round-5 docs head (abtrees/r5head, de436c6).
set -o pipefail
cd /root/repo && source tools/gpu.sh
out r5/mid
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_mlkem.py \
  tests/test_gpu_schedule.py tests/test_gpu_ordering.py > $O/tests_mlkem_mid.log 2>&1 || { tail -30 $O/tests_mlkem_mid.log; exit 1; }
tail -3 $O/tests_mlkem_mid.log
out r5/mid/ab14 && abx 3 new=default old=tree:abtrees/r5head -- --log2-batch 14 --steps 60 --warmup 10 --no-profile || exit 1
out r5/mid/ab15 && abx 3 new=default old=tree:abtrees/r5head -- --log2-batch 15 --steps 40 --warmup 5 --no-profile || exit 1
out r5/mid/ab16 && abx 3 new=default old=tree:abtrees/r5head -- --log2-batch 16 --steps 30 --warmup 5 --no-profile || exit 1
out r5/mid/prof && for lb in 14 15; do bench new_$lb --log2-batch $lb --steps 60 --warmup 10 --no-cpu || exit 1; done
echo mid_done
