# round 6: same-box interleaved A/B of the multi-role schedule (--streams 0, the
# default) against the serial one (--streams 1, one kernel per launch) at 2^20 and 2^16, ML-KEM-768
# enc+dec, on HEAD.  Run it on two boxes (TAG=a, TAG=b).
set -o pipefail
cd /root/repo && source tools/gpu.sh && out r6/sched${TAG:-}
abx 4 s0_2p20=default s1_2p20=default,--streams,1 -- --steps 20 --warmup 5 &&
abx 4 s0_2p16=default,--log2-batch,16 s1_2p16=default,--log2-batch,16,--streams,1 -- --steps 50 --warmup 10 &&
python3 - $O/abx.jsonl <<'PY'
import json, sys, statistics
rows = [json.loads(l) for l in open(sys.argv[1])]
by = {}
for r in rows:
    by.setdefault(r["tag"], []).append(r["value"])
for t, v in by.items():
    print(t, "median %.4g" % statistics.median(v), "runs", " ".join("%.4g" % x for x in v))
PY
