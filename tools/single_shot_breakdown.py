#!/usr/bin/env python3
"""Where one handshake's latency goes on the GPU library (ML-KEM-768, n = 1):
  oqs_*      : the reference call pattern (a new qrkem.oqs.KeyEncapsulation per call, bytes in/out)
  host_*     : BatchKEM host-array call (one C-ABI call: staging, H2D, kernel, D2H, sync)
  device_*   : BatchKEM device-tensor call + torch.cuda.synchronize() (no PCIe)
  kernel_*   : the kernel(s) alone, HIP events on the launch stream (qrk_ctx_profile)
Median microseconds over N calls; one JSON line."""
import json
import statistics
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "quantum-resistant-p2p_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
from qrkem import oqs  # noqa: E402
from qrkem.batch import BatchKEM  # noqa: E402

ALG, N = sys.argv[1] if len(sys.argv) > 1 else "ML-KEM-768", 200
med = lambda v: round(statistics.median(v) * 1e6, 1)  # noqa: E731
out = {}
kem = oqs.KeyEncapsulation(ALG)
pk = kem.generate_keypair()
sk = kem.export_secret_key()
t = {"oqs_keypair": [], "oqs_encaps": [], "oqs_decaps": []}
for _ in range(N):
    t0 = time.perf_counter(); kem.generate_keypair(); t["oqs_keypair"].append(time.perf_counter() - t0)
    t0 = time.perf_counter(); c, ss = oqs.KeyEncapsulation(ALG).encap_secret(pk); t["oqs_encaps"].append(time.perf_counter() - t0)
    t0 = time.perf_counter(); oqs.KeyEncapsulation(ALG, sk).decap_secret(c); t["oqs_decaps"].append(time.perf_counter() - t0)
eng = BatchKEM(ALG, device=0)
hpk = np.frombuffer(pk, np.uint8).reshape(1, -1).copy()
hsk = np.frombuffer(sk, np.uint8).reshape(1, -1).copy()
hct = np.frombuffer(c, np.uint8).reshape(1, -1).copy()
kc = np.zeros((1, eng.kp_coins), np.uint8)
for k in ("host_keypair", "host_encaps", "host_decaps"):
    t[k] = []
for _ in range(N):
    t0 = time.perf_counter(); eng.keypair(coins=kc); t["host_keypair"].append(time.perf_counter() - t0)
    t0 = time.perf_counter(); eng.encaps(hpk); t["host_encaps"].append(time.perf_counter() - t0)
    t0 = time.perf_counter(); eng.decaps(hsk, hct); t["host_decaps"].append(time.perf_counter() - t0)
dpk, dsk, dct = (torch.from_numpy(a).cuda() for a in (hpk, hsk, hct))
dkc = torch.from_numpy(kc).cuda()
dec = torch.zeros((1, eng.enc_coins), dtype=torch.uint8, device="cuda")
torch.cuda.synchronize()
for k in ("device_keypair", "device_encaps", "device_decaps"):
    t[k] = []
for _ in range(N):
    t0 = time.perf_counter(); eng.keypair(coins=dkc); torch.cuda.synchronize(); t["device_keypair"].append(time.perf_counter() - t0)
    t0 = time.perf_counter(); eng.encaps(dpk, coins=dec); torch.cuda.synchronize(); t["device_encaps"].append(time.perf_counter() - t0)
    t0 = time.perf_counter(); eng.decaps(dsk, dct); torch.cuda.synchronize(); t["device_decaps"].append(time.perf_counter() - t0)
out = {k: med(v) for k, v in t.items()}
eng.profile(True)
for _ in range(N):
    eng.keypair(coins=dkc); eng.encaps(dpk, coins=dec); eng.decaps(dsk, dct)
torch.cuda.synchronize()
prof = eng.profile_read()
out["kernel_us"] = {k: round(ms * 1e3 / cnt, 1) for k, (ms, cnt) in prof.items()}
print(json.dumps({"alg": ALG, "single_shot_median_us": out}))
