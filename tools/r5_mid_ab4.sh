# round 5, mid-size batches: Decaps' G(m' || h) + PRFs in one role beside the fix-up (k_g_prf) at
# chunks <= 2^15, against the separate k_g_decaps launch (variant gprf0, QRK_GPRF=0)
set -o pipefail
cd /root/repo && source tools/gpu.sh
out r5/mid4
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_mlkem.py \
  tests/test_gpu_schedule.py tests/test_gpu_ordering.py > $O/tests_mlkem_mid4.log 2>&1 || { tail -30 $O/tests_mlkem_mid4.log; exit 1; }
tail -2 $O/tests_mlkem_mid4.log
for lb in 14 15; do
  out r5/mid4/ab$lb && abx 4 gprf=default sep=gprf0 -- --log2-batch $lb --steps 60 --warmup 10 --no-profile || exit 1
done
out r5/mid4/prof && for lb in 14 15; do bench gprf_$lb --log2-batch $lb --steps 60 --warmup 10 --no-cpu || exit 1; done
echo mid4_done
