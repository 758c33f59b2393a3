# round 6 final build: the whole GPU suite, smoke, the default bench line, rocprofv3 trace +
# FETCH/WRITE + SQ passes of the bench command, single-shot latency, the handshake line, and the
# mid-size per-call rates without per-launch events (--no-profile)
set -o pipefail
cd /root/repo && source tools/gpu.sh && out r6/final
SUITE_TIMEOUT=1500 suite tests || exit 1
smoke || exit 1
bench bench_default && cut -c1-300 $O/bench_default.json || exit 1
prof mlkem768 || exit 1
sq mlkem768 || exit 1
PROF_STEPS=1 sq mlkem768_serial --streams 1 || exit 1
timeout -k 10 300 python3 -u tools/single_shot_breakdown.py ML-KEM-768 > $O/single_shot_breakdown.jsonl || exit 1
bench handshake_mlkem768 --mode handshake --no-cpu || exit 1
for b in 14 15 16 20; do
  bench noprof_2p$b --log2-batch $b --steps 50 --warmup 10 --no-cpu --no-profile || exit 1
done
echo r6_final_done
