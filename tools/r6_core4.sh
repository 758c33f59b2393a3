# round 6: ML-KEM-1024 encrypt / re-encryption core at 3 waves per SIMD (168 VGPRs; the Decaps form
# spills 16 B) against the default (174 / 176 VGPRs, 2 waves per SIMD): enc+dec at 2^20 and the
# half-tampered decaps config, interleaved on one box
set -o pipefail
cd /root/repo && source tools/gpu.sh && out r6/core4
abx 3 def=default,--alg,ML-KEM-1024 w3=core4w3,--alg,ML-KEM-1024 def_t=default,--alg,ML-KEM-1024,--mode,decaps-tampered w3_t=core4w3,--alg,ML-KEM-1024,--mode,decaps-tampered -- --steps 10 --warmup 2 || exit 1
python3 - $O/abx.jsonl <<'PY'
import json, sys, statistics
by = {}
for l in open(sys.argv[1]):
    r = json.loads(l); by.setdefault(r["tag"], []).append(r)
for t, rs in by.items():
    print(t, "median %.4g" % statistics.median(x["value"] for x in rs), {k: round(v, 3) for k, v in rs[0]["kernels_timed_region"].items()})
PY
