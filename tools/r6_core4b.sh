# round 6: ML-KEM-1024 Encaps core at 3 waves per SIMD (no spill), the Decaps core unchanged --
# ML-KEM tests, then interleaved against the previous head (head6) at 2^20 enc+dec and tampered decaps
set -o pipefail
cd /root/repo && source tools/gpu.sh && out r6/core4b
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_mlkem.py tests/test_gpu_fullsize.py -k "1024 or mlkem" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
abx 4 new=default,--alg,ML-KEM-1024 head=head6,--alg,ML-KEM-1024 new_t=default,--alg,ML-KEM-1024,--mode,decaps-tampered head_t=head6,--alg,ML-KEM-1024,--mode,decaps-tampered -- --steps 10 --warmup 2 || exit 1
python3 - $O/abx.jsonl <<'PY'
import json, sys, statistics
by = {}
for l in open(sys.argv[1]):
    r = json.loads(l); by.setdefault(r["tag"], []).append(r)
for t, rs in by.items():
    print(t, "median %.4g" % statistics.median(x["value"] for x in rs), " ".join("%.4g" % x["value"] for x in rs), {k: round(v, 3) for k, v in rs[0]["kernels_timed_region"].items()})
PY
