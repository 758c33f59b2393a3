# round 6: KeyGen's H(ek) kernel (k_back_keygen, 127 VGPRs with the next-block prefetch) without the
# prefetch (backnopf) against HEAD (head7), handshake driver at 2^20, interleaved
set -o pipefail
cd /root/repo && source tools/gpu.sh && out r6/backpf
abx 3 nopf=backnopf head=head7 -- --mode handshake --steps 10 --warmup 3 || exit 1
python3 - $O/abx.jsonl <<'PY'
import json, sys, statistics
by = {}
for l in open(sys.argv[1]):
    r = json.loads(l); by.setdefault(r["tag"], []).append(r)
for t, rs in by.items():
    print(t, "median %.4g" % statistics.median(x["value"] for x in rs), " ".join("%.4g" % x["value"] for x in rs), {k: round(v, 3) for k, v in rs[0]["kernels_timed_region"].items() if "keygen" in k})
PY
