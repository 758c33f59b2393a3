# round 6: pipelined single-shot KeyGen with failure semantics + agent acquire (default), expanded-key
# reuse in the handshake driver -- GPU tests, then interleaved A/Bs: OQS latency against the round-4
# kernel (kgmulti) and the round-5 pipelined kernel (r5pipe, built from the round-5 head), and the
# handshake driver at 2^20 against the round-5 library (r5pipe)
set -o pipefail
cd /root/repo && O=gpurun_out/r6/kg${TAG:-} && mkdir -p $O
source tools/gpu.sh && out r6/kg${TAG:-}
V=quantum-resistant-p2p_amd/qrkem/variants
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_mlkem.py tests/test_gpu_ordering.py tests/test_gpu_wire.py tests/test_gpu_handshake.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2 3; do
  timeout -k 10 120 python -u tools/single_shot_breakdown.py ML-KEM-768 | sed 's/^{/{"variant": "pipe_acq", /' >> $O/ab_kg.jsonl || exit $?
  QRKEM_LIBRARY=$V/libqrkem_kgmulti.so timeout -k 10 120 python -u tools/single_shot_breakdown.py ML-KEM-768 | sed 's/^{/{"variant": "multi", /' >> $O/ab_kg.jsonl || exit $?
  QRKEM_LIBRARY=$V/libqrkem_r5pipe.so timeout -k 10 120 python -u tools/single_shot_breakdown.py ML-KEM-768 | sed 's/^{/{"variant": "r5pipe", /' >> $O/ab_kg.jsonl || exit $?
done
python - $O/ab_kg.jsonl <<'PY'
import json,sys
for l in open(sys.argv[1]):
    d=json.loads(l); s=d['single_shot_median_us']
    print(d['variant'], 'oqs_keypair', s['oqs_keypair'], 'host_keypair', s['host_keypair'], 'oqs_enc', s['oqs_encaps'], 'oqs_dec', s['oqs_decaps'])
PY
abx 3 hs_r6=default hs_r5=r5pipe -- --mode handshake --steps 10 --warmup 3 && cat $O/abx.jsonl | cut -c1-120
probe ss_service ss_service_probe.hip && cat $O/ss_service.txt
