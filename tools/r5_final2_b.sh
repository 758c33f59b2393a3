# round 5, second final build: one bench line per BASELINE.json config and SURVEY 8f mode (gpu.sh
# sweep), then the mid-size chunk lines
set -o pipefail
cd /root/repo && source tools/gpu.sh && out r5/sweep
sweep || exit 1
for lb in 16 15 14; do bench mlkem768_2p$lb --log2-batch $lb --steps 40 --warmup 5 || exit 1; done
echo final2_b_done
