#!/usr/bin/env python3
"""ML-KEM-768 encaps+decaps time per batch (device tensors, median of R) at batch sizes around the
one-launch / batched-schedule boundary (QRK_SMALL_MAX).  Run once per library build:
    QRKEM_LIBRARY=<lib> python3 tools/small_crossover.py <tag>"""
import json
import statistics
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "quantum-resistant-p2p_amd"))
import torch  # noqa: E402
from qrkem.batch import BatchKEM  # noqa: E402

tag = sys.argv[1] if len(sys.argv) > 1 else "default"
eng = BatchKEM("ML-KEM-768", device=0)
out = {}
for n in (64, 256, 512, 1024, 2048, 4096, 8192, 16384, 65536):
    kc = eng.bench_coins(n, 96, 7, 0)
    pk, sk = eng.keypair(coins=kc[:, :64].contiguous())
    ec = kc[:, 64:].contiguous()
    for _ in range(3):
        ct, ss = eng.encaps(pk, coins=ec)
        eng.decaps(sk, ct)
    torch.cuda.synchronize()
    ts = []
    for _ in range(15 if n <= 8192 else 5):
        t0 = time.perf_counter()
        ct, ss = eng.encaps(pk, coins=ec)
        ss2 = eng.decaps(sk, ct)
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    assert bool((ss == ss2).all())
    m = statistics.median(ts)
    out[n] = {"us": round(m * 1e6, 1), "per_s": round(n / m)}
print(json.dumps({"tag": tag, "encdec": out}))
