# round 5, second final build: single-shot OQS latency (qrkem.oqs and the stock wrapper)
set -o pipefail
cd /root/repo && source tools/gpu.sh && out r5/final2
timeout -k 10 300 python3 -u tools/single_shot_latency.py > $O/single_shot_latency.json || exit 1
cat $O/single_shot_latency.json
