"""HIP HQC-128/192/256 parity vs the oracle, through the C ABI (libqrkem.so).

Bar: byte-exact pk / sk / ct / ss and identical decaps return codes for every index
(integer work).  Checker: the C oracle (oracle/src/hqc.c), held to the pure-Python
restatement and the frozen vectors in tests/test_hqc_oracle.py.  PARITY UNPINNED against
liboqs itself (no HQC KATs offline).  Sizes are ragged; the chunked path is covered.
"""
import hashlib
import json
from pathlib import Path

import numpy as np
import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu

ALGS = ["HQC-128", "HQC-192", "HQC-256"]
GOLD = json.loads((Path(__file__).parent / "golden" / "hqc.json").read_text())


@pytest.fixture(scope="module")
def engines():
    from qrkem.batch import BatchKEM
    return {a: BatchKEM(a, device=0) for a in ALGS}


def _dev(a):
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


def _host(t):
    torch.cuda.synchronize()
    return t.cpu().numpy()


def _coins(alg, n, seed):
    import oracle as orc
    s = orc.sizes(alg)
    return orc.bench_coins(n, s["keypair_coins"], seed=seed), orc.bench_coins(n, s["encaps_coins"], seed=seed + 1)


@pytest.mark.parametrize("alg", ALGS)
def test_golden_records(engines, alg):
    eng = engines[alg]
    recs = GOLD[alg]["records"]
    kc = np.stack([np.frombuffer(bytes.fromhex(r["kp_coins"]), np.uint8) for r in recs])
    ec = np.stack([np.frombuffer(bytes.fromhex(r["enc_coins"]), np.uint8) for r in recs])
    pk, sk = eng.keypair(coins=_dev(kc))
    ct, ss = eng.encaps(pk, coins=_dev(ec))
    ss2, st = eng.decaps(sk, ct, return_status=True)
    pk, sk, ct, ss, ss2, st = map(_host, (pk, sk, ct, ss, ss2, st))
    for i, r in enumerate(recs):
        assert hashlib.sha256(pk[i].tobytes()).hexdigest() == r["pk"]
        assert hashlib.sha256(sk[i].tobytes()).hexdigest() == r["sk"]
        assert hashlib.sha256(ct[i].tobytes()).hexdigest() == r["ct"]
        assert ss[i].tobytes().hex() == r["ss"] and ss2[i].tobytes().hex() == r["ss"]
    assert list(st) == [0] * len(recs)
    bad = ct.copy()
    for i in range(len(recs)):
        bit = (13 * i + 5) % (8 * bad.shape[1])
        bad[i, bit // 8] ^= 1 << (bit % 8)
    tss, tst = eng.decaps(_dev(sk), _dev(bad), return_status=True)
    tss, tst = _host(tss), _host(tst)
    for i, r in enumerate(recs):
        assert tss[i].tobytes().hex() == r["tampered_ss"]
    assert list(tst) == [-1] * len(recs)


@pytest.mark.parametrize("alg", ALGS)
@pytest.mark.parametrize("n", [1, 67])
def test_roundtrip_matches_oracle(engines, alg, n):
    import oracle as orc
    eng = engines[alg]
    kc, ec = _coins(alg, n, 500 + n)
    pk, sk = eng.keypair(coins=_dev(kc))
    ct, ss = eng.encaps(pk, coins=_dev(ec))
    ss2 = eng.decaps(sk, ct)
    pk, sk, ct, ss, ss2 = map(_host, (pk, sk, ct, ss, ss2))
    opk, osk = orc.batch_keypair(alg, kc)
    assert np.array_equal(pk, opk)
    assert np.array_equal(sk, osk)
    oct_, oss = orc.batch_encaps(alg, opk, ec)
    assert np.array_equal(ct, oct_)
    assert np.array_equal(ss, oss)
    assert np.array_equal(ss2, oss)


@pytest.mark.parametrize("alg", ALGS)
def test_mixed_tampered_batch(engines, alg):
    """Every other ciphertext has one bit flipped (a different byte each time, u, v and salt
    alike): ss and the per-record return code equal the oracle's."""
    import oracle as orc
    eng = engines[alg]
    n = 40
    kc, ec = _coins(alg, n, 77)
    opk, osk = orc.batch_keypair(alg, kc)
    oct_, oss = orc.batch_encaps(alg, opk, ec)
    bad = oct_.copy()
    L = bad.shape[1]
    for i in range(1, n, 2):
        pos = (i * 997) % L
        bad[i, pos] ^= 1 << (i % 8)
    ref_ss, ref_st = orc.batch_decaps(alg, osk, bad, with_status=True)
    ss, st = eng.decaps(_dev(osk), _dev(bad), return_status=True)
    assert np.array_equal(_host(ss), ref_ss)
    assert np.array_equal(_host(st), ref_st)
    assert list(ref_st) == [0, -1] * (n // 2)
    # host-buffer path, same answers
    hss, hst = eng.decaps(osk, bad, return_status=True)
    assert np.array_equal(hss, ref_ss) and np.array_equal(hst, ref_st)


@pytest.mark.parametrize("alg", ALGS)
def test_stray_bits_above_n(engines, alg):
    """Malformed inputs with bits above X^(n-1): the pk's s (Encaps) and the ct's u (Decaps)."""
    import oracle as orc
    eng = engines[alg]
    n = 8
    kc, ec = _coins(alg, n, 91)
    opk, osk = orc.batch_keypair(alg, kc)
    s = orc.sizes(alg)
    nb = s["pk"] - 40
    bpk = opk.copy()
    bpk[:, -1] |= 0xE0
    ct, ss = eng.encaps(_dev(bpk), coins=_dev(ec))
    oct_, oss = orc.batch_encaps(alg, bpk, ec)
    assert np.array_equal(_host(ct), oct_) and np.array_equal(_host(ss), oss)
    gct, _ = orc.batch_encaps(alg, opk, ec)
    bct = gct.copy()
    bct[:, nb - 1] |= 0x80
    ref_ss, ref_st = orc.batch_decaps(alg, osk, bct, with_status=True)
    dss, dst = eng.decaps(_dev(osk), _dev(bct), return_status=True)
    assert np.array_equal(_host(dss), ref_ss) and np.array_equal(_host(dst), ref_st)
    assert (ref_st == -1).all()


def test_chunked_batch(engines):
    """n larger than the context chunk: several launches, equal to the oracle."""
    import oracle as orc
    from qrkem.batch import BatchKEM
    alg = "HQC-128"
    eng = BatchKEM(alg, device=0, chunk=128)
    n = 300
    kc, ec = _coins(alg, n, 31)
    pk, sk = eng.keypair(coins=_dev(kc))
    ct, ss = eng.encaps(pk, coins=_dev(ec))
    ss2 = eng.decaps(sk, ct)
    opk, _ = orc.batch_keypair(alg, kc)
    oct_, oss = orc.batch_encaps(alg, opk, ec)
    assert np.array_equal(_host(pk), opk)
    assert np.array_equal(_host(ct), oct_)
    assert np.array_equal(_host(ss), oss) and np.array_equal(_host(ss2), oss)


@pytest.mark.parametrize("level,alg", [(1, "HQC-128"), (3, "HQC-192"), (5, "HQC-256")])
def test_plugin_single_shot(level, alg):
    """HQCKeyExchange as the reference uses it (key_exchange.py:189-309): fresh objects per
    call, OS coins; a rejected ciphertext raises, as liboqs's error return does via oqs.py."""
    from qrkem.key_exchange import HQCKeyExchange
    kem = HQCKeyExchange(security_level=level)
    assert kem.variant == alg and kem.name == f"HQC (Level {level})"
    pk, sk = kem.generate_keypair()
    ct, ss = kem.encapsulate(pk)
    assert kem.decapsulate(sk, ct) == ss and len(ss) == 64
    bad = bytearray(ct)
    bad[100] ^= 4
    with pytest.raises(RuntimeError):
        kem.decapsulate(sk, bytes(bad))


def _r_for(sup, n):
    """random words r_i with i + floor(r_i (n - i) / 2^32) = sup_i (needs i <= sup_i < n)"""
    r = [-(-((s - i) << 32) // (n - i)) for i, s in enumerate(sup)]
    assert all(i + ((x * (n - i)) >> 32) == s for i, (x, s) in enumerate(zip(r, sup)))
    return r


@pytest.mark.parametrize("alg", ALGS)
def test_supports_duplicate_removal(engines, alg):
    """qrk_hqc_supports on supports crafted to collide (value duplicates, index collisions, a
    chain through every index) vs the spec's serial loop (hqc_spec.remove_duplicates)."""
    import random

    import hqc_spec as H
    p = H.params(alg)
    n = p["n"]
    rng = random.Random(n)
    for kind, w in ((0, p["w"]), (1, p["wr"])):
        sups = [
            [i + rng.randrange(4) for i in range(w)],
            [w + 5] * w,
            [i + 1 for i in range(w - 1)] + [w - 1],
            [rng.randrange(i, 2 * w) for i in range(w)],
            [rng.randrange(i, n) for i in range(w)],
            [n - 1] * w,
            list(range(w)),
        ]
        r = np.array([_r_for(s, n) for s in sups], dtype=np.uint32)
        got = _host(engines[alg].hqc_supports(_dev(r.view(np.int32)), kind)).view(np.uint32)
        for s, g in zip(sups, got):
            assert list(g) == H.remove_duplicates(s)


@pytest.mark.parametrize("alg", ALGS)
@pytest.mark.parametrize("n", [256, 257])
def test_coop_lane_boundary(engines, alg, n):
    """n = 256 runs the seedexpanders and the K hash on the wave-cooperative sponges
    (QRK_HQC_COOP_MAX), n = 257 on the lane kernels: byte-exact vs the oracle, tampered
    ciphertexts with the oracle's status."""
    import oracle as orc
    eng = engines[alg]
    kc, ec = _coins(alg, n, 6000 + n)
    pk, sk = eng.keypair(coins=_dev(kc))
    ct, ss = eng.encaps(pk, coins=_dev(ec))
    ct_h = _host(ct)
    bad = ct_h.copy()
    bad[1::2, 11] ^= 0x04
    ss2 = eng.decaps(sk, ct)
    ss3, st3 = eng.decaps(sk, _dev(bad), return_status=True)
    pk, sk, ss, ss2, ss3, st3 = map(_host, (pk, sk, ss, ss2, ss3, st3))
    opk, osk = orc.batch_keypair(alg, kc)
    assert np.array_equal(pk, opk) and np.array_equal(sk, osk)
    oct_, oss = orc.batch_encaps(alg, opk, ec)
    assert np.array_equal(ct_h, oct_) and np.array_equal(ss, oss) and np.array_equal(ss2, oss)
    ref_ss, ref_st = orc.batch_decaps(alg, osk, bad, with_status=True)
    assert np.array_equal(ss3, ref_ss) and np.array_equal(st3, ref_st)
