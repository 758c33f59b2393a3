# round 6: where the single-shot KeyGen's 3.1 us launch call goes -- the launch-cost probe, then
# interleaved OQS latency of the default build against a build that launches k_keygen_pipe through
# hipModuleLaunchKernel on a cached hipFunction_t (modl), and the host traces of both
set -o pipefail
cd /root/repo && source tools/gpu.sh && out r6/launch
V=quantum-resistant-p2p_amd/qrkem/variants
probe launch_cost launch_cost_probe.hip && cat $O/launch_cost.txt
for r in 1 2 3; do
  timeout -k 10 120 python -u tools/single_shot_breakdown.py ML-KEM-768 | sed 's/^{/{"variant": "default", /' >> $O/ab_modl.jsonl || exit $?
  QRKEM_LIBRARY=$V/libqrkem_modl.so timeout -k 10 120 python -u tools/single_shot_breakdown.py ML-KEM-768 | sed 's/^{/{"variant": "modl", /' >> $O/ab_modl.jsonl || exit $?
done
QRKEM_LIBRARY=$V/libqrkem_htrace.so timeout -k 10 120 python -u tools/host_trace.py > $O/htrace_default.jsonl || exit $?
QRKEM_LIBRARY=$V/libqrkem_htmodl.so timeout -k 10 120 python -u tools/host_trace.py > $O/htrace_modl.jsonl || exit $?
python - $O/ab_modl.jsonl <<'PY'
import json,sys
for l in open(sys.argv[1]):
    d=json.loads(l); s=d['single_shot_median_us']
    print(d['variant'], 'oqs_keypair', s['oqs_keypair'], 'host_keypair', s['host_keypair'])
PY
head -1 $O/htrace_default.jsonl; head -1 $O/htrace_modl.jsonl
