"""The auto schedule -- with the split SampleNTT / encrypt-core pipeline when it is built in
(QRK_SPLIT in csrc/mlkem.hip, off by default) -- against the serial schedule and the
C oracle.

At full chunks (auto stream mode, n >= 2^18, chunk a multiple of 64 * parts) k_xof runs in parts
on the context's side stream while the main stream runs the front hash, the PRFs and the encrypt
core part by part.  n = 300000 makes the last part ragged (74976 of 75008).  Every output of the
split schedule must equal the serial schedule's (qrk_ctx_set_streams(1), no side stream, no split)
byte for byte over the whole batch -- KeyGen, Encaps, and Decaps with half the ciphertexts tampered
(the re-encryption compare and implicit rejection) -- and a sample around every part boundary must
equal the oracle.  Each stage is compared on its own, so a failure names the stage and counts the
mismatching rows per part.
"""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu

N = 300000
PARTS = 4


def _boundary_idx(n, parts=PARTS):
    cq = ((n + 63) // 64 * 64) // parts
    idx = [0, 1, n - 1]
    for q in range(1, parts):
        idx += [q * cq - 2, q * cq - 1, q * cq, q * cq + 1]
    return np.unique(np.array([i for i in idx if 0 <= i < n]))


def _rows_per_part(a, b, n=N, parts=PARTS):
    bad = torch.nonzero((a != b).any(dim=1)).flatten().cpu()
    cq = ((n + 63) // 64 * 64) // parts
    return [int(((bad >= q * cq) & (bad < (q + 1) * cq)).sum()) for q in range(parts)], bad[:8].tolist()


@pytest.mark.parametrize("alg", ["ML-KEM-768", "ML-KEM-1024"])
def test_split_back_to_back(alg):
    """KeyGen -> Encaps -> tamper -> Decaps on one auto-schedule context with no host
    synchronisation in between (calls overlap through the streams), then the serial schedule."""
    from qrkem.batch import BatchKEM
    eng = BatchKEM(alg, device=0)
    coins = eng.bench_coins(N, 96, seed=400 + len(alg))
    kc, ec = coins[:, :64].contiguous(), coins[:, 64:].contiguous()
    pk, sk = eng.keypair(coins=kc)
    ct, ss = eng.encaps(pk, coins=ec)
    bad = ct.clone()
    eng.tamper(bad, seed=78, mode=2)
    ss2 = eng.decaps(sk, bad)
    torch.cuda.synchronize()
    ser = BatchKEM(alg, device=0)
    ser.set_streams(1)
    pk_s, sk_s = ser.keypair(coins=kc)
    ct_s, ss_s = ser.encaps(pk_s, coins=ec)
    ss2_s = ser.decaps(sk_s, bad)
    torch.cuda.synchronize()
    stages = {"pk": _rows_per_part(pk, pk_s), "sk": _rows_per_part(sk, sk_s), "ct": _rows_per_part(ct, ct_s),
              "ss": _rows_per_part(ss, ss_s), "ss2": _rows_per_part(ss2, ss2_s)}
    assert all(sum(v[0]) == 0 for v in stages.values()), stages
    del pk, sk, ct, ss, bad, ss2, pk_s, sk_s, ct_s, ss_s, ss2_s, coins, kc, ec
    eng.close()
    ser.close()
    torch.cuda.empty_cache()


@pytest.mark.parametrize("alg", ["ML-KEM-768", "ML-KEM-1024"])
def test_split_schedule_equals_serial_and_oracle(alg):
    import oracle as orc
    from qrkem.batch import BatchKEM
    eng = BatchKEM(alg, device=0)  # auto schedule: split at this size
    ser = BatchKEM(alg, device=0)
    ser.set_streams(1)  # serial schedule: no side stream, no split
    coins = eng.bench_coins(N, 96, seed=300 + len(alg))
    kc, ec = coins[:, :64].contiguous(), coins[:, 64:].contiguous()

    pk, sk = eng.keypair(coins=kc)
    pk_s, sk_s = ser.keypair(coins=kc)
    torch.cuda.synchronize()
    assert torch.equal(pk, pk_s), ("keypair pk", _rows_per_part(pk, pk_s))
    assert torch.equal(sk, sk_s), ("keypair sk", _rows_per_part(sk, sk_s))

    ct, ss = eng.encaps(pk, coins=ec)
    ct_s, ss_s = ser.encaps(pk, coins=ec)
    torch.cuda.synchronize()
    assert torch.equal(ct, ct_s), ("encaps ct", _rows_per_part(ct, ct_s))
    assert torch.equal(ss, ss_s), ("encaps ss", _rows_per_part(ss, ss_s))

    bad = ct.clone()
    eng.tamper(bad, seed=77, mode=2)
    flip = (bad != ct).any(dim=1)
    ss2 = eng.decaps(sk, bad)
    ss2_s = ser.decaps(sk, bad)
    torch.cuda.synchronize()
    assert torch.equal(ss2_s[~flip], ss[~flip]), "serial decaps of untampered rows"
    assert torch.equal(ss2, ss2_s), ("decaps ss", _rows_per_part(ss2, ss2_s))
    assert not bool((ss2[flip] == ss[flip]).all(dim=1).any())

    idx = _boundary_idx(N)
    ti = torch.from_numpy(idx).cuda()
    kc_h, ec_h, ct_h, ss_h, bad_h, ss2_h = (t.index_select(0, ti).cpu().numpy()
                                            for t in (kc, ec, ct, ss, bad, ss2))
    opk, osk = orc.batch_keypair(alg, np.ascontiguousarray(kc_h))
    oct_, oss = orc.batch_encaps(alg, opk, np.ascontiguousarray(ec_h))
    assert np.array_equal(ct_h, oct_) and np.array_equal(ss_h, oss)
    assert np.array_equal(ss2_h, orc.batch_decaps(alg, osk, np.ascontiguousarray(bad_h)))
    del pk, sk, ct, ss, bad, ss2, pk_s, sk_s, ct_s, ss_s, ss2_s, coins, kc, ec
    eng.close()
    ser.close()
    torch.cuda.empty_cache()
