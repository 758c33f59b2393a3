#!/usr/bin/env python3
"""Phase times inside HQC-128 k_hqc_enc_mul / k_hqc_decode under full load (2^16 batch), from a
-DQRK_HQC_TRACE=1 build (workgroup QRK_HQC_TRACE_WG stamps its phase boundaries):
    tools/build_variant.sh hqctrace -DQRK_HQC_TRACE=1
    QRKEM_LIBRARY=quantum-resistant-p2p_amd/qrkem/variants/libqrkem_hqctrace.so python3 tools/hqc_trace.py
Microseconds after the workgroup's first stamp, median over R runs."""
import ctypes
import json
import statistics
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "quantum-resistant-p2p_amd"))
import torch  # noqa: E402
from qrkem._native import LIB  # noqa: E402
from qrkem.batch import BatchKEM  # noqa: E402

ALG = sys.argv[1] if len(sys.argv) > 1 else "HQC-128"
N, R = 1 << 16, 7
fn = LIB.qrk_dbg_hqc_trace
fn.argtypes = [ctypes.POINTER(ctypes.c_ulonglong)]
ENC = {1: "A: h, s doubled, supports, GF tables", 24: "B: start", 25: "B: dedupe r1 (wave 0)",
       26: "B: RS parity (wave 3)", 2: "B: barrier", 3: "C: sparse_dense (own)",
       4: "C: barrier (all classes)", 5: "prod_combine", 6: "message assembly", 7: "stores"}
DEC = {17: "u doubled, ct staging, supports", 18: "dedupe", 19: "sparse_dense (own)", 20: "prod_combine",
       21: "RM(1,7) decoding", 22: "stores"}


def read():
    buf = (ctypes.c_ulonglong * 32)()
    assert fn(buf) == 0
    return list(buf)


eng = BatchKEM(ALG, device=0)
pk, sk = eng.keypair(n=N)
ct, ss = eng.encaps(pk)
torch.cuda.synchronize()
acc = {("enc", k): [] for k in ENC} | {("reenc", k): [] for k in ENC} | {("dec", k): [] for k in DEC}
for _ in range(R):
    eng.encaps(pk)
    torch.cuda.synchronize()
    t = read()
    for k in ENC:
        acc[("enc", k)].append((t[k] - t[0]) / 100.0)
    eng.decaps(sk, ct)
    torch.cuda.synchronize()
    t = read()
    for k in ENC:
        kk = k + 4 if k >= 24 else 8 + k
        acc[("reenc", k)].append((t[kk] - t[8]) / 100.0)
    for k in DEC:
        acc[("dec", k)].append((t[k] - t[16]) / 100.0)
out = {"enc_mul": {f"{k}:{v}": statistics.median(acc[("enc", k)]) for k, v in ENC.items()},
       "enc_mul_reenc": {f"{k}:{v}": statistics.median(acc[("reenc", k)]) for k, v in ENC.items()},
       "decode": {f"{k}:{v}": statistics.median(acc[("dec", k)]) for k, v in DEC.items()}}
print(json.dumps({"alg": ALG, "batch": N, "phase_us_from_wg_start": out}))
