# round 6, VERDICT r5 item 8: HQC-128 Encaps product with wider windows (WPTE 9, NBTE 64: 10 reads per
# 9 words instead of 6 per 5) -- the HQC-128 tests on each variant, then interleaved A/Bs at 2^16
# against the default (WPTE 5, NBTE 128, 8 waves / SIMD). Variants: hqc_e9 (8 waves, 132 / 100 B
# spilled), hqc_e9w6 (6 waves, 44 / 48 B spilled), hqc_e9w5 (5 waves, no spill in the bench kernel)
set -o pipefail
cd /root/repo && source tools/gpu.sh && out r6/hqcwin
V=quantum-resistant-p2p_amd/qrkem/variants
for t in hqc_e9 hqc_e9w6 hqc_e9w5; do
  QRKEM_LIBRARY=$V/libqrkem_$t.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
    tests/test_gpu_hqc.py -k "128" > $O/tests_$t.log 2>&1 || { tail -20 $O/tests_$t.log; exit 1; }
  echo "$t $(tail -1 $O/tests_$t.log)"
done
abx 3 w5=default e9=hqc_e9 e9w6=hqc_e9w6 e9w5=hqc_e9w5 -- --alg HQC-128 --steps 20 --warmup 3 --no-cpu || exit 1
python3 - $O/abx.jsonl <<'PY'
import json, sys, statistics
by = {}
for l in open(sys.argv[1]):
    r = json.loads(l); by.setdefault(r["tag"], []).append(r)
for t, rs in by.items():
    ks = rs[0]["kernels_timed_region"]
    em = [x["kernels_timed_region"].get("k_hqc_enc_mul", {}).get("avg_ms") for x in rs]
    print(t, "median %.4g" % statistics.median(x["value"] for x in rs), "enc_mul ms", em, "roofline", rs[0].get("roofline", {}).get("frac"))
PY
echo hqcwin_done
