"""The split SampleNTT / encrypt-core pipeline (QRK_SPLIT in csrc/mlkem.hip) against the serial
schedule and the C oracle.

At full chunks (auto stream mode, n >= 2^18, chunk a multiple of 64 * parts) k_xof runs in parts
on the context's side stream while the main stream runs the front hash, the PRFs and the encrypt
core part by part.  n = 300000 makes the last part ragged (74976 of 75008).  Every output of the
split schedule must equal the serial schedule's (qrk_ctx_set_streams(1), no side stream, no split)
byte for byte over the whole batch, and a sample around every part boundary must equal the oracle,
for Encaps (encrypt core MODE 0) and for Decaps with half the ciphertexts tampered (MODE 1, the
re-encryption compare and implicit rejection).
"""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu

N = 300000


def _boundary_idx(n, parts=4):
    cq = ((n + 63) // 64 * 64) // parts
    idx = [0, 1, n - 1]
    for q in range(1, parts):
        idx += [q * cq - 2, q * cq - 1, q * cq, q * cq + 1]
    return np.unique(np.array([i for i in idx if 0 <= i < n]))


@pytest.mark.parametrize("alg", ["ML-KEM-768", "ML-KEM-1024"])
def test_split_schedule_equals_serial_and_oracle(alg):
    import oracle as orc
    from qrkem.batch import BatchKEM
    eng = BatchKEM(alg, device=0)
    coins = eng.bench_coins(N, 96, seed=300 + len(alg))
    kc, ec = coins[:, :64].contiguous(), coins[:, 64:].contiguous()
    pk, sk = eng.keypair(coins=kc)
    ct, ss = eng.encaps(pk, coins=ec)  # auto schedule: split
    bad = ct.clone()
    eng.tamper(bad, seed=77, mode=2)
    flip = (bad != ct).any(dim=1)
    ss2 = eng.decaps(sk, bad)
    torch.cuda.synchronize()
    assert bool((ss2[~flip] == ss[~flip]).all())
    assert not bool((ss2[flip] == ss[flip]).all(dim=1).any())

    ser = BatchKEM(alg, device=0)
    ser.set_streams(1)  # serial schedule: no side stream, no split
    ct_s, ss_s = ser.encaps(pk, coins=ec)
    ss2_s = ser.decaps(sk, bad)
    torch.cuda.synchronize()
    assert torch.equal(ct, ct_s) and torch.equal(ss, ss_s) and torch.equal(ss2, ss2_s)

    idx = _boundary_idx(N)
    ti = torch.from_numpy(idx).cuda()
    kc_h, ec_h, ct_h, ss_h, bad_h, ss2_h = (t.index_select(0, ti).cpu().numpy()
                                            for t in (kc, ec, ct, ss, bad, ss2))
    opk, osk = orc.batch_keypair(alg, np.ascontiguousarray(kc_h))
    oct_, oss = orc.batch_encaps(alg, opk, np.ascontiguousarray(ec_h))
    assert np.array_equal(ct_h, oct_) and np.array_equal(ss_h, oss)
    assert np.array_equal(ss2_h, orc.batch_decaps(alg, osk, np.ascontiguousarray(bad_h)))
    del pk, sk, ct, ss, bad, ss2, ct_s, ss_s, ss2_s, coins, kc, ec
    eng.close()
    ser.close()
    torch.cuda.empty_cache()
