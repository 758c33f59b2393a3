# round 6: the whole GPU suite and smoke on HEAD, the default bench line, the schedule A/B on a
# second box (TAG=b), and the mid-size per-launch times (serial schedule, one kernel per launch)
# at 2^14 / 2^15 next to the multi-role per-call rates at 2^14 / 2^15 / 2^16
set -o pipefail
cd /root/repo && source tools/gpu.sh && out r6/c
SUITE_TIMEOUT=1500 suite tests || exit 1
smoke || exit 1
bench bench_default && cat $O/bench_default.json | cut -c1-400 || exit 1
TAG=b bash tools/r6_sched.sh || exit 1
out r6/c
for b in 14 15; do
  bench mid_serial_2p$b --log2-batch $b --streams 1 --steps 50 --warmup 10 --no-cpu || exit 1
done
for b in 14 15 16; do
  bench mid_multi_2p$b --log2-batch $b --steps 50 --warmup 10 --no-cpu || exit 1
done
echo r6_c_done
