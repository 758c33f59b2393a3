# round 5: lane-pair sponge fronts at chunks <= 2^15 -- parity, then interleaved A/B at 2^14 / 2^15 / 2^16
set -o pipefail
cd /root/repo && source tools/gpu.sh && out r5/pair${TAG:-}
suite tests/test_gpu_mlkem.py tests/test_gpu_schedule.py || exit 1
for lb in 14 15; do
  out r5/pair${TAG:-}/b$lb
  abx 3 pair=default prio=pairprio off=pairoff -- --log2-batch $lb --steps 60 --warmup 10 --no-profile || exit 1
done
out r5/pair${TAG:-}/b16 && abx 2 pair=default off=pairoff -- --log2-batch 16 --steps 30 --warmup 5 --no-profile || exit 1
