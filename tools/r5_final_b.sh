# round 5 final build, part B: same-box interleaved A/B against the round-4 head (abtrees/r4head,
# commit c157b14) at 2^20 / 2^16 / 2^15 / 2^14 handshakes per call, then the profiles
set -o pipefail
cd /root/repo && source tools/gpu.sh
out r5/final/ab20 && abx 4 r5=default r4=tree:abtrees/r4head -- --steps 20 --warmup 5 --no-profile || exit 1
out r5/final/ab16 && abx 3 r5=default r4=tree:abtrees/r4head -- --log2-batch 16 --steps 30 --warmup 5 --no-profile || exit 1
out r5/final/ab15 && abx 3 r5=default r4=tree:abtrees/r4head -- --log2-batch 15 --steps 40 --warmup 5 --no-profile || exit 1
out r5/final/ab14 && abx 3 r5=default r4=tree:abtrees/r4head -- --log2-batch 14 --steps 60 --warmup 10 --no-profile || exit 1
out r5/final && prof mlkem768 || exit 1
sq mlkem768 || exit 1
timeout -k 10 300 python3 -u tools/single_shot_latency.py > $O/single_shot_latency.json || exit 1
for a in ML-KEM-768 ML-KEM-512 ML-KEM-1024; do timeout -k 10 120 python3 -u tools/single_shot_breakdown.py $a >> $O/single_shot_breakdown.jsonl || exit 1; done
echo final_b_done
