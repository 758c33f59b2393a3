#!/usr/bin/env python3
"""Where the host side of one single-shot OQS call goes (a -DQRK_HOST_TRACE=1 build):
    tools/build_variant.sh htrace -DQRK_HOST_TRACE=1
    QRKEM_LIBRARY=quantum-resistant-p2p_amd/qrkem/variants/libqrkem_htrace.so python3 tools/host_trace.py
Stamps (abi.cpp HT(i)): 0 single() entry, 1 context locked, 2 inputs staged in the pinned mirror,
3 run_batch ready to launch, 4 launch call returned, 5 run_batch returned (its end event recorded),
6 completion ticket seen, 7 outputs copied out + mirror wiped, 9 single() returns.  Also the Python
call time around it.  Median microseconds over N calls, one JSON line per operation."""
import ctypes
import json
import statistics
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "quantum-resistant-p2p_amd"))
from qrkem import oqs  # noqa: E402
from qrkem._native import LIB  # noqa: E402

fn = LIB.qrk_dbg_host_trace
fn.argtypes = [ctypes.POINTER(ctypes.c_longlong)]
ALG, N = sys.argv[1] if len(sys.argv) > 1 else "ML-KEM-768", 300
kem = oqs.KeyEncapsulation(ALG)
pk = kem.generate_keypair()
sk = kem.export_secret_key()
c, _ = oqs.KeyEncapsulation(ALG).encap_secret(pk)
names = {1: "lock", 2: "stage_inputs", 3: "run_batch_setup", 4: "launch_call", 5: "end_event_record",
         6: "kernel_to_ticket_seen", 7: "copy_out_wipe", 9: "return"}
for op in ("keypair", "encaps", "decaps"):
    d = {k: [] for k in names}
    py = []
    for _ in range(N):
        t0 = time.perf_counter()
        if op == "keypair":
            kem.generate_keypair()
        elif op == "encaps":
            oqs.KeyEncapsulation(ALG).encap_secret(pk)
        else:
            oqs.KeyEncapsulation(ALG, sk).decap_secret(c)
        py.append(time.perf_counter() - t0)
        b = (ctypes.c_longlong * 16)()
        fn(b)
        prev = 0
        for k in sorted(names):
            d[k].append((b[k] - b[prev]) / 1e3)
            prev = k
    out = {names[k]: round(statistics.median(v), 2) for k, v in d.items()}
    out["python_call_total"] = round(statistics.median(py) * 1e6, 1)
    print(json.dumps({"alg": ALG, "op": op, "host_phase_us": out}))
