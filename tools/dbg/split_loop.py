#!/usr/bin/env python3
"""Race hunt for the split schedule: the tests/test_gpu_split.py sequence (fresh context, KeyGen,
Encaps, tamper, Decaps on the auto schedule) repeated in one process, mismatches vs the serial
schedule per part printed per iteration.  usage: split_loop.py alg iters"""
import sys
import time
import torch
sys.path.insert(0, "quantum-resistant-p2p_amd")
from qrkem.batch import BatchKEM

alg, iters, n = sys.argv[1], int(sys.argv[2]), 300000
ser = BatchKEM(alg, device=0)
ser.set_streams(1)
cq = ((n + 63) // 64 * 64) // 4
def parts(b):
    idx = torch.nonzero(b).flatten().cpu()
    return [int(((idx >= q * cq) & (idx < (q + 1) * cq)).sum()) for q in range(4)]
for it in range(iters):
    eng = BatchKEM(alg, device=0)
    coins = eng.bench_coins(n, 96, seed=300 + it)
    kc, ec = coins[:, :64].contiguous(), coins[:, 64:].contiguous()
    pk, sk = eng.keypair(coins=kc)
    ct, ss = eng.encaps(pk, coins=ec)
    bad = ct.clone()
    eng.tamper(bad, seed=77 + it, mode=2)
    ss2 = eng.decaps(sk, bad)
    torch.cuda.synchronize()
    pk_s, sk_s = ser.keypair(coins=kc)
    ct_s, ss_s = ser.encaps(pk_s, coins=ec)
    ss2_s = ser.decaps(sk_s, bad)
    torch.cuda.synchronize()
    r = {"pk": parts((pk != pk_s).any(1)), "sk": parts((sk != sk_s).any(1)), "ct": parts((ct != ct_s).any(1)),
         "ss": parts((ss != ss_s).any(1)), "ss2": parts((ss2 != ss2_s).any(1))}
    print(it, r, flush=True)
    eng.close()
    del eng, pk, sk, ct, ss, bad, ss2, pk_s, sk_s, ct_s, ss_s, ss2_s, coins, kc, ec
    torch.cuda.empty_cache()
