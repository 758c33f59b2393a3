"""BASELINE.json's full sizes on the GPU, through size-independent properties.

configs[1]: ML-KEM-512/768/1024, 2^20 handshakes in one batch on one MI355X -- every
ss_enc == ss_dec, and a stride sample of the batch (first/last tiles, chunk-ish
boundaries, every 2^14-th index) byte-exact vs the C oracle.
configs[4]: ML-KEM-1024 decaps of 2^20 ciphertexts, about half of them tampered with
one flipped bit -- untampered indices give ss_enc, tampered ones never do, and the
sample equals the oracle's implicit-rejection key J(z || c).
The oracle only checks the sample; the whole batch runs through libqrkem.so.
"""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu

N = 1 << 20


def _sample_idx(n):
    return np.unique(np.r_[0:64, n // 2 - 3:n // 2 + 3, 0:n:1 << 14, n - 64:n])


@pytest.mark.parametrize("alg", ["ML-KEM-512", "ML-KEM-768", "ML-KEM-1024"])
def test_full_batch_roundtrip_and_sample(alg):
    import oracle as orc
    from qrkem.batch import BatchKEM
    eng = BatchKEM(alg, device=0)
    coins = eng.bench_coins(N, 96, seed=20 + len(alg))
    kc, ec = coins[:, :64].contiguous(), coins[:, 64:].contiguous()
    pk, sk = eng.keypair(coins=kc)
    ct, ss = eng.encaps(pk, coins=ec)
    ss2 = eng.decaps(sk, ct)
    torch.cuda.synchronize()
    assert bool((ss == ss2).all())
    # no two handshakes share a key (distinct coins -> distinct ss)
    assert torch.unique(ss[:, :8].contiguous().view(torch.int64).flatten()).numel() == N
    idx = _sample_idx(N)
    ti = torch.from_numpy(idx).cuda()
    pk_h, sk_h, ct_h, ss_h, kc_h, ec_h = (t.index_select(0, ti).cpu().numpy()
                                          for t in (pk, sk, ct, ss, kc, ec))
    opk, osk = orc.batch_keypair(alg, np.ascontiguousarray(kc_h))
    oct_, oss = orc.batch_encaps(alg, opk, np.ascontiguousarray(ec_h))
    assert np.array_equal(pk_h, opk) and np.array_equal(sk_h, osk)
    assert np.array_equal(ct_h, oct_) and np.array_equal(ss_h, oss)
    del pk, sk, ct, ss, ss2, coins, kc, ec
    torch.cuda.empty_cache()


def test_full_batch_tampered_decaps_1024():
    import oracle as orc
    from qrkem.batch import BatchKEM
    alg = "ML-KEM-1024"
    eng = BatchKEM(alg, device=0)
    coins = eng.bench_coins(N, 96, seed=4)
    kc, ec = coins[:, :64].contiguous(), coins[:, 64:].contiguous()
    pk, sk = eng.keypair(coins=kc)
    ct, ss = eng.encaps(pk, coins=ec)
    bad = ct.clone()
    eng.tamper(bad, seed=1024, mode=2)
    flip = (bad != ct).any(dim=1)
    frac = flip.float().mean().item()
    assert 0.49 < frac < 0.51
    ss2 = eng.decaps(sk, bad)
    torch.cuda.synchronize()
    assert bool((ss2[~flip] == ss[~flip]).all())
    assert not bool((ss2[flip] == ss[flip]).all(dim=1).any())
    idx = _sample_idx(N)
    ti = torch.from_numpy(idx).cuda()
    sk_h, bad_h, ss2_h = (t.index_select(0, ti).cpu().numpy() for t in (sk, bad, ss2))
    want = orc.batch_decaps(alg, np.ascontiguousarray(sk_h), np.ascontiguousarray(bad_h))
    assert np.array_equal(ss2_h, want)
    del pk, sk, ct, ss, bad, ss2, coins, kc, ec
    torch.cuda.empty_cache()


FRODO_SEC = {"640": 16, "976": 24, "1344": 32}


@pytest.mark.parametrize("alg", ["FrodoKEM-640-SHAKE", "FrodoKEM-976-SHAKE", "FrodoKEM-1344-SHAKE",
                                 "FrodoKEM-640-AES", "FrodoKEM-976-AES", "FrodoKEM-1344-AES"])
def test_frodo_bench_batch_roundtrip_tamper_and_sample(alg):
    """configs[3] at the bench's FrodoKEM batch (2^16 in one chunk): every ss_enc == ss_dec,
    a one-bit tamper on every other ciphertext always rejects, and a sample of KeyGen /
    Encaps / tampered Decaps is byte-exact vs the C oracle.  The sample holds every
    1024-th index, both sides of the 2^15 midpoint and the tail (the indices a round-1
    scratch run flagged, DESIGN.md section 8: a harness coin-width error, not a kernel one)."""
    import oracle as orc
    from qrkem.batch import BatchKEM
    n = 1 << 16
    sec = FRODO_SEC[alg.split("-")[1]]
    eng = BatchKEM(alg, device=0)
    kpl = 2 * sec + 16  # s || seedSE || z, then mu
    coins = eng.bench_coins(n, kpl + sec, seed=640 + sec)
    kc, ec = coins[:, :kpl].contiguous(), coins[:, kpl:].contiguous()
    pk, sk = eng.keypair(coins=kc)
    ct, ss = eng.encaps(pk, coins=ec)
    ss2 = eng.decaps(sk, ct)
    bad = ct.clone()
    eng.tamper(bad, seed=sec, mode=2)
    flip = (bad != ct).any(dim=1)
    ss3 = eng.decaps(sk, bad)
    torch.cuda.synchronize()
    assert bool((ss == ss2).all())
    assert 0.48 < flip.float().mean().item() < 0.52
    assert bool((ss3[~flip] == ss[~flip]).all())
    assert not bool((ss3[flip] == ss[flip]).all(dim=1).any())
    idx = np.unique(np.r_[0:4, n // 2 - 2:n // 2 + 2, 0:n:1 << 10, 1023:n:1 << 10, n - 4:n])
    ti = torch.from_numpy(idx).cuda()
    pk_h, sk_h, ct_h, ss_h, kc_h, ec_h, bad_h, ss3_h = (
        t.index_select(0, ti).cpu().numpy() for t in (pk, sk, ct, ss, kc, ec, bad, ss3))
    opk, osk = orc.batch_keypair(alg, np.ascontiguousarray(kc_h), 16)
    bad_pk = idx[(pk_h != opk).any(axis=1)]
    bad_sk = idx[(sk_h != osk).any(axis=1)]
    assert bad_pk.size == 0 and bad_sk.size == 0, (bad_pk[:8], bad_sk[:8])
    oct_, oss = orc.batch_encaps(alg, opk, np.ascontiguousarray(ec_h), 16)
    assert np.array_equal(ct_h, oct_) and np.array_equal(ss_h, oss)
    assert np.array_equal(ss3_h, orc.batch_decaps(alg, osk, np.ascontiguousarray(bad_h), 16))
    del pk, sk, ct, ss, ss2, ss3, bad, coins, kc, ec
    torch.cuda.empty_cache()


@pytest.mark.parametrize("alg", ["HQC-128", "HQC-192", "HQC-256"])
def test_hqc_bench_batch_roundtrip_tamper_and_sample(alg):
    """HQC at the bench's 2^16 batch: every ss_enc == ss_dec with status 0, a one-bit tamper
    on every other ciphertext gives status -1 and a different key on exactly those indices,
    and a sample of KeyGen / Encaps / tampered Decaps (key and status) is byte-exact vs the
    C oracle."""
    import oracle as orc
    from qrkem.batch import BatchKEM
    n = 1 << 16
    eng = BatchKEM(alg, device=0)
    kpl, encl = eng.kp_coins, eng.enc_coins
    # bench_coins squeezes one SHAKE256 block (<= 136 B, whole words): one draw per role
    kc = eng.bench_coins(n, (kpl + 7) // 8 * 8, seed=128)[:, :kpl].contiguous()
    ec = eng.bench_coins(n, (encl + 7) // 8 * 8, seed=129)[:, :encl].contiguous()
    coins = None
    pk, sk = eng.keypair(coins=kc)
    ct, ss = eng.encaps(pk, coins=ec)
    ss2, st2 = eng.decaps(sk, ct, return_status=True)
    bad = ct.clone()
    eng.tamper(bad, seed=3, mode=2)
    flip = (bad != ct).any(dim=1)
    ss3, st3 = eng.decaps(sk, bad, return_status=True)
    torch.cuda.synchronize()
    assert bool((ss == ss2).all()) and bool((st2 == 0).all())
    assert 0.48 < flip.float().mean().item() < 0.52
    assert bool((ss3[~flip] == ss[~flip]).all()) and bool((st3[~flip] == 0).all())
    assert not bool((ss3[flip] == ss[flip]).all(dim=1).any())
    assert bool((st3[flip] == -1).all())
    idx = np.unique(np.r_[0:4, n // 2 - 2:n // 2 + 2, 0:n:1 << 12, n - 4:n])
    ti = torch.from_numpy(idx).cuda()
    pk_h, sk_h, ct_h, ss_h, kc_h, ec_h, bad_h, ss3_h, st3_h = (
        t.index_select(0, ti).cpu().numpy() for t in (pk, sk, ct, ss, kc, ec, bad, ss3, st3))
    opk, osk = orc.batch_keypair(alg, np.ascontiguousarray(kc_h), 8)
    oct_, oss = orc.batch_encaps(alg, opk, np.ascontiguousarray(ec_h), 8)
    assert np.array_equal(pk_h, opk) and np.array_equal(sk_h, osk)
    assert np.array_equal(ct_h, oct_) and np.array_equal(ss_h, oss)
    oss3, ost3 = orc.batch_decaps(alg, osk, np.ascontiguousarray(bad_h), 8, with_status=True)
    assert np.array_equal(ss3_h, oss3) and np.array_equal(st3_h, ost3)
    del pk, sk, ct, ss, ss2, ss3, bad, coins, kc, ec
    torch.cuda.empty_cache()
