# round 6: HQC seedexpander streams and K hash on lane pairs (<= QRK_HQC_PAIR_MAX = 2^17 handshakes):
# the HQC GPU tests, then interleaved A/Bs against the lane-only build (hqclane) at 2^16 for every
# level, and the threshold at 2^17 / 2^18 for HQC-128 against a pairs-everywhere build (hqcpairall)
set -o pipefail
cd /root/repo && source tools/gpu.sh && out r6/hqc
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_hqc.py tests/test_gpu_fullsize.py -k "hqc or HQC" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
abx 3 pair128=default,--alg,HQC-128 lane128=hqclane,--alg,HQC-128 pair192=default,--alg,HQC-192 lane192=hqclane,--alg,HQC-192 pair256=default,--alg,HQC-256 lane256=hqclane,--alg,HQC-256 -- --steps 20 --warmup 3 || exit 1
abx 2 lane128_2p17=hqclane,--alg,HQC-128,--log2-batch,17 pair128_2p17=default,--alg,HQC-128,--log2-batch,17 lane128_2p18=hqclane,--alg,HQC-128,--log2-batch,18 pair128_2p18=hqcpairall,--alg,HQC-128,--log2-batch,18 -- --steps 10 --warmup 2 || exit 1
python3 - $O/abx.jsonl <<'PY'
import json, sys, statistics
by = {}
for l in open(sys.argv[1]):
    r = json.loads(l); by.setdefault(r["tag"], []).append(r)
for t, rs in by.items():
    print(t, "median %.4g" % statistics.median(x["value"] for x in rs), {k: round(v, 4) for k, v in rs[0]["kernels_timed_region"].items()})
PY
