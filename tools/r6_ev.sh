# round 6: the context's I/O stream records its last-use event lazily (abi.cpp LastUse) -- the
# whole GPU suite on that build, then the OQS single-shot latency interleaved against the library
# built from the previous head (variants/libqrkem_preev.so), four rounds on one box
set -o pipefail
cd /root/repo && source tools/gpu.sh && out r6/ev
V=quantum-resistant-p2p_amd/qrkem/variants
SUITE_TIMEOUT=1500 suite tests || exit 1
for r in 1 2 3 4; do
  timeout -k 10 120 python -u tools/single_shot_breakdown.py ML-KEM-768 | sed 's/^{/{"variant": "lazy_ev", /' >> $O/ab_ev.jsonl || exit $?
  QRKEM_LIBRARY=$V/libqrkem_preev.so timeout -k 10 120 python -u tools/single_shot_breakdown.py ML-KEM-768 | sed 's/^{/{"variant": "prev_head", /' >> $O/ab_ev.jsonl || exit $?
done
python - $O/ab_ev.jsonl <<'PY'
import json,sys
for l in open(sys.argv[1]):
    d=json.loads(l); s=d['single_shot_median_us']
    print(d['variant'], 'oqs kp/enc/dec', s['oqs_keypair'], s['oqs_encaps'], s['oqs_decaps'], 'host', s['host_keypair'], s['host_encaps'], s['host_decaps'])
PY
echo ev_done
