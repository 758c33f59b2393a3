#!/usr/bin/env python3
"""Phase times inside the ML-KEM single-shot kernels (n = 1), from a -DQRK_SS_TRACE=1 build:
    tools/build_variant.sh sstrace -DQRK_SS_TRACE=1
    QRKEM_LIBRARY=quantum-resistant-p2p_amd/qrkem/variants/libqrkem_sstrace.so python3 tools/single_shot_trace.py
Each phase is microseconds after the kernel's first stamp (100 MHz wall clock), median of N calls."""
import ctypes
import json
import statistics
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "quantum-resistant-p2p_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
from qrkem._native import LIB  # noqa: E402
from qrkem.batch import BatchKEM  # noqa: E402

ALG, N = sys.argv[1] if len(sys.argv) > 1 else "ML-KEM-768", 100
fn = LIB.qrk_dbg_ss_trace
fn.argtypes = [ctypes.POINTER(ctypes.c_ulonglong)]
MARKS = {
    # k_keygen_multi (n = 1): one workgroup per PRF / SampleNTT item, the last to count in finishes
    # k_keygen_pipe (n = 1 host-pointer calls, the default there): t = 0 is the collector workgroup's start
    "keypair": {1: "PRF item 0 published", 7: "H wave: G done", 10: "SampleNTT A[0][0] block 1",
                11: "block 2", 12: "block 3", 2: "A[0][0] done", 22: "t wave: s_hat, e_hat loaded",
                8: "H block 0 starts", 13: "H block 1 starts", 9: "H block 2 starts", 14: "H block 3 starts",
                3: "t_hat_0 done", 19: "row 1 t_hat published", 5: "t_hat_1.. copied in", 4: "H(ek) done",
                6: "done (wipe, flags reset)"},
    "encaps": {1: "H(ek)+G done", 3: "wave 1 SampleNTT done", 2: "wave 0 PRF + NTT(y_0) done", 4: "sync", 7: "u rows done"},
    "decaps": {8: "decrypt done", 9: "G done", 12: "wave 2 SampleNTT done", 10: "wave 2 PRF done", 4: "rows start",
               11: "J done", 6: "rows done, v + Kbar ready", 7: "select done"},
}


def read():
    buf = (ctypes.c_ulonglong * 32)()
    assert fn(buf) == 0
    return list(buf)


eng = BatchKEM(ALG, device=0)
pk, sk = eng.keypair(n=1)
ct, ss = eng.encaps(pk)
torch.cuda.synchronize()
out = {}
for op in ("keypair", "encaps", "decaps"):
    acc = {k: [] for k in MARKS[op]}
    mhz = []
    for _ in range(N):
        if op == "keypair":  # host coins: the host-pointer path runs the pipelined KeyGen (k_keygen_pipe)
            eng.keypair(coins=np.random.default_rng(_).integers(0, 256, (1, 64), dtype=np.uint8))
        elif op == "encaps":
            eng.encaps(pk)
        else:
            eng.decaps(sk, ct)
        torch.cuda.synchronize()
        t = read()
        for k in MARKS[op]:
            acc[k].append((t[k] - t[0]) / 100.0)
        if op == "encaps":
            mhz.append((t[21] - t[20]) / ((t[1] - t[0]) / 100.0))
    out[op] = {f"{k}:{v}": round(statistics.median(acc[k]), 2) for k, v in MARKS[op].items()}
    if op == "encaps":  # shader clock over H(ek) + G: clock64 cycles / wall-clock time
        out[op]["shader_MHz_during_H_G"] = round(statistics.median(mhz), 1)
print(json.dumps({"alg": ALG, "phase_us_from_kernel_start": out}))
