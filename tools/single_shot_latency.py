#!/usr/bin/env python3
"""Latency of the reference's call pattern on the GPU library: one handshake per
OQS_KEM_* call through qrkem.oqs (the drop-in for vendor/oqs.py:318, 348, 372).
Prints one JSON line: microseconds per keypair / encaps / decaps (median of N calls)."""
import json
import statistics
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "quantum-resistant-p2p_amd"))
from qrkem import oqs  # noqa: E402

out = {}
# "(stock wrapper)": the handle's fields read on every construction, as the reference's unmodified
# vendor/oqs.py does (oqs.py:273-280), instead of qrkem.oqs's per-mechanism cache
for alg in ("ML-KEM-768", "ML-KEM-768 (stock wrapper)", "FrodoKEM-640-AES"):
    stock = alg.endswith("(stock wrapper)")
    name = alg.split(" ")[0]
    if stock:
        _KE = oqs.KeyEncapsulation

        def KE(*a, **k):
            oqs._ATTRS.clear()
            return _KE(*a, **k)
    else:
        KE = oqs.KeyEncapsulation
    kem = KE(name)
    pk = kem.generate_keypair()
    sk = kem.export_secret_key()
    N = 200 if name.startswith("ML") else 50
    t = {"keypair": [], "encaps": [], "decaps": []}
    for _ in range(N):
        t0 = time.perf_counter(); kem.generate_keypair(); t["keypair"].append(time.perf_counter() - t0)
        t0 = time.perf_counter(); c, ss = KE(name).encap_secret(pk); t["encaps"].append(time.perf_counter() - t0)
        t0 = time.perf_counter(); ss2 = KE(name, sk).decap_secret(c); t["decaps"].append(time.perf_counter() - t0)
        assert ss == ss2
    out[alg] = {k: round(statistics.median(v) * 1e6, 1) for k, v in t.items()}
print(json.dumps({"single_shot_median_us": out}))
