# round 5, mid-size batches, second pass: J split (QRK_JSPLIT) and rho read from the keys
# (QRK_DIRECT_RHO_MAX) separately and together, against the round-5 docs head (abtrees/r5head)
set -o pipefail
cd /root/repo && source tools/gpu.sh
out r5/mid2
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_mlkem.py \
  tests/test_gpu_schedule.py tests/test_gpu_ordering.py > $O/tests_mlkem_mid2.log 2>&1 || { tail -30 $O/tests_mlkem_mid2.log; exit 1; }
tail -2 $O/tests_mlkem_mid2.log
for lb in 14 15; do
  out r5/mid2/ab$lb && abx 3 both=default js=js dr=dr old=tree:abtrees/r5head -- --log2-batch $lb --steps 60 --warmup 10 --no-profile || exit 1
done
out r5/mid2/prof && for lb in 14 15; do bench both_$lb --log2-batch $lb --steps 60 --warmup 10 --no-cpu || exit 1; done
echo mid2_done
