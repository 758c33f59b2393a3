"""Debug: FrodoKEM KeyGen B (unpacked from pk) on the GPU vs the oracle, diff pattern."""
import sys
from pathlib import Path
import numpy as np
import torch
R = Path(__file__).resolve().parents[2]
sys.path[:0] = [str(R / "quantum-resistant-p2p_amd"), str(R / "oracle")]
import oracle as orc
from qrkem.batch import BatchKEM

alg = sys.argv[1] if len(sys.argv) > 1 else "FrodoKEM-640-SHAKE"
n_, logq = {"640": (640, 15), "976": (976, 16), "1344": (1344, 16)}[alg.split("-")[1]]
sec = {"640": 16, "976": 24, "1344": 32}[alg.split("-")[1]]
kc = orc.bench_coins(2, 2 * sec + 16, seed=301)
eng = BatchKEM(alg, device=0)
pk, sk = eng.keypair(coins=torch.from_numpy(kc).cuda())
torch.cuda.synchronize()
pk = pk.cpu().numpy()
opk, _ = orc.batch_keypair(alg, kc)


def unpack(p):
    bits = np.unpackbits(p[16:])
    v = bits[: n_ * 8 * logq].reshape(-1, logq)
    return (v * (1 << np.arange(logq - 1, -1, -1))).sum(axis=1).reshape(n_, 8)


for h in range(2):
    g, o = unpack(pk[h]), unpack(opk[h])
    d = (g.astype(np.int64) - o) % (1 << logq)
    bad = np.argwhere(d != 0)
    print("hs", h, "seedA equal", bool((pk[h, :16] == opk[h, :16]).all()), "bad entries", len(bad), "of", d.size)
    if len(bad):
        rows = np.unique(bad[:, 0]); ks = np.unique(bad[:, 1])
        print(" bad rows", rows[:20], "... count", len(rows), " bad k", ks)
        print(" sample diffs", [(int(r), int(k), int(d[r, k]), int(g[r, k]), int(o[r, k])) for r, k in bad[:12]])
np.savez("gpurun_out/kgdiff.npz", pk=pk, opk=opk, kc=kc)
