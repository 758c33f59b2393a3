#!/usr/bin/env python3
"""BASELINE.json configs[0] (CPU plumbing, no GPU): ML-KEM-768 KeyGen/Encaps/Decaps of the 1024
NIST-KAT-DRBG handshakes through the C oracle (liboqs is absent: its stand-in), single thread,
checked against the committed golden digest (tests/golden/kat_mlkem768.json).  One JSON line."""
import hashlib
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "oracle"))
import oracle as orc  # noqa: E402

ALG, N = "ML-KEM-768", 1024
_, kc, ec = orc.kat_coins(N, 64, 32)
t0 = time.perf_counter()
pk, sk = orc.batch_keypair(ALG, kc, threads=1)
ct, ss = orc.batch_encaps(ALG, pk, ec, threads=1)
ss2 = orc.batch_decaps(ALG, sk, ct, threads=1)
dt = time.perf_counter() - t0
assert (ss == ss2).all()
g = json.load(open(ROOT / "tests" / "golden" / "kat_mlkem.json"))[ALG]["digests"]
h = {k: hashlib.sha256(a.tobytes()).hexdigest() for k, a in (("pk", pk), ("sk", sk), ("ct", ct), ("ss", ss))}
print(json.dumps({"config": "BASELINE.json configs[0]", "alg": ALG, "handshakes": N, "threads": 1,
                  "seconds": round(dt, 3), "handshakes_per_s": round(N / dt, 1),
                  "golden_digests_match": h == g, "cpu": open("/proc/cpuinfo").read().split("model name")[1].split("\n")[0].strip(": ")}))
