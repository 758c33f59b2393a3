"""HIP FrodoKEM (SHAKE and AES Gen(A)) parity vs the oracle, through the C ABI (libqrkem.so).

Bar: byte-exact pk / sk / ct / ss for every index (integer work).  The oracle
(oracle/src/frodo.c, pinned to the Python restatement oracle/py/frodo_spec.py via
tests/golden/kat_frodo.json) is the checker.  Sizes are ragged (not multiples of
the 64-handshake scratch tile or the 256-handshake Gen(A) sub-chunk).
"""
import hashlib
import json

import numpy as np
import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu

ALGS = ["FrodoKEM-640-SHAKE", "FrodoKEM-976-SHAKE", "FrodoKEM-1344-SHAKE",
        "FrodoKEM-640-AES", "FrodoKEM-976-AES", "FrodoKEM-1344-AES"]
SEC = {a: {"640": 16, "976": 24, "1344": 32}[a.split("-")[1]] for a in ALGS}
GOLDEN_ALGS = ALGS


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
    kpl, encl = 2 * SEC[alg] + 16, SEC[alg]  # s || seedSE || z (len_z = 16), mu
    c = orc.bench_coins(n, kpl + encl, seed=seed)
    return np.ascontiguousarray(c[:, :kpl]), np.ascontiguousarray(c[:, kpl:])


@pytest.mark.parametrize("alg", ALGS)
@pytest.mark.parametrize("n", [1, 3, 70])
def test_roundtrip_matches_oracle(engines, alg, n):
    import oracle as orc
    eng = engines[alg]
    kc, ec = _coins(alg, n, 300 + n)
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
def test_encaps_decaps_on_oracle_keys(engines, alg):
    """Encaps / Decaps alone (keys from the oracle), crossing the 256-handshake sub-chunk."""
    import oracle as orc
    eng = engines[alg]
    n = 300 if alg.startswith("FrodoKEM-640") else 97
    kc, ec = _coins(alg, n, 8)
    opk, osk = orc.batch_keypair(alg, kc, 8)
    oct_, oss = orc.batch_encaps(alg, opk, ec, 8)
    ct, ss = eng.encaps(_dev(opk), coins=_dev(ec))
    assert np.array_equal(_host(ct), oct_)
    assert np.array_equal(_host(ss), oss)
    assert np.array_equal(_host(eng.decaps(_dev(osk), _dev(oct_))), oss)


@pytest.mark.parametrize("alg", ALGS)
def test_tampered_implicit_rejection(engines, alg):
    """Flipped bits anywhere in ct (B' part and C part) -> ss = H(ct || s), as the oracle."""
    import oracle as orc
    eng = engines[alg]
    n = 40
    kc, ec = _coins(alg, n, 99)
    opk, osk = orc.batch_keypair(alg, kc, 8)
    oct_, oss = orc.batch_encaps(alg, opk, ec, 8)
    bad = oct_.copy()
    rng = np.random.default_rng(7)
    flip = rng.random(n) < 0.5
    L = bad.shape[1]
    for j, i in enumerate(np.nonzero(flip)[0]):
        # alternate between the packed B' region and the trailing C region
        lo = 0 if j % 2 == 0 else L - 120  # packed C is 120 (640) / 128 bytes
        bit = int(rng.integers(8 * lo, 8 * L))
        bad[i, bit // 8] ^= 1 << (bit % 8)
    ss = _host(eng.decaps(_dev(osk), _dev(bad)))
    want = orc.batch_decaps(alg, osk, bad, 8)
    assert np.array_equal(ss, want)
    assert np.array_equal(ss[~flip], oss[~flip])
    assert not np.any(np.all(ss[flip] == oss[flip], axis=1))


@pytest.mark.parametrize("alg", GOLDEN_ALGS)
def test_kat_drbg_records_match_golden(engines, golden_dir, alg):
    """NIST-KAT-DRBG coins, digests of the Python restatement (tests/golden/kat_frodo.json)."""
    import oracle as orc
    g = json.loads((golden_dir / "kat_frodo.json").read_text())[alg]
    n = g["count"]
    _, kc, ec = orc.kat_coins(n, g["kp_coins"], g["enc_coins"])
    eng = engines[alg]
    pk, sk = eng.keypair(coins=_dev(kc))
    ct, ss = eng.encaps(pk, coins=_dev(ec))
    ss2 = eng.decaps(sk, ct)
    pk, sk, ct, ss, ss2 = map(_host, (pk, sk, ct, ss, ss2))
    assert np.array_equal(ss, ss2)
    for name, arr in (("pk", pk), ("sk", sk), ("ct", ct), ("ss", ss)):
        assert hashlib.sha256(arr.tobytes()).hexdigest() == g["digests"][name], name


@pytest.mark.parametrize("alg", ["FrodoKEM-640-SHAKE", "FrodoKEM-640-AES"])
def test_multichunk_640(engines, alg):
    """More handshakes than one Frodo chunk (2^14 cap lowered via set_chunk): ss_enc == ss_dec
    everywhere, a sample byte-exact vs the oracle."""
    import oracle as orc
    from qrkem.batch import BatchKEM
    n = 1200
    eng = BatchKEM(alg, device=0, chunk=512)
    coins = eng.bench_coins(n, 64, seed=42)
    kc, ec = coins[:, :48].contiguous(), coins[:, 48:].contiguous()
    pk, sk = eng.keypair(coins=kc)
    ct, ss = eng.encaps(pk, coins=ec)
    ss2 = eng.decaps(sk, ct)
    torch.cuda.synchronize()
    assert bool((ss == ss2).all())
    idx = np.r_[0:4, 510:515, 1020:1026, n - 3:n]
    pk_h, sk_h, ct_h, ss_h = (t.cpu().numpy()[idx] for t in (pk, sk, ct, ss))
    kc_h, ec_h = kc.cpu().numpy()[idx], ec.cpu().numpy()[idx]
    opk, osk = orc.batch_keypair(alg, np.ascontiguousarray(kc_h), 8)
    oct_, oss = orc.batch_encaps(alg, opk, np.ascontiguousarray(ec_h), 8)
    assert np.array_equal(pk_h, opk) and np.array_equal(sk_h, osk)
    assert np.array_equal(ct_h, oct_) and np.array_equal(ss_h, oss)


@pytest.mark.parametrize("alg", ["FrodoKEM-640-SHAKE", "FrodoKEM-640-AES", "FrodoKEM-976-SHAKE"])
@pytest.mark.parametrize("n", [256, 257])
def test_coop_lane_boundary(engines, alg, n):
    """n = 256 runs H(pk), the SE stream and ss = H(ct || k) on the wave-cooperative sponges
    (QRK_FR_COOP_MAX), n = 257 on the lane-per-handshake kernels: both byte-exact vs the oracle,
    including tampered-ciphertext Decaps (implicit rejection through H(ct' || s))."""
    import oracle as orc
    eng = engines[alg]
    kc, ec = _coins(alg, n, 4000 + n)
    pk, sk = eng.keypair(coins=_dev(kc))
    ct, ss = eng.encaps(pk, coins=_dev(ec))
    ct_h = _host(ct)
    bad = ct_h.copy()
    bad[1::2, 7] ^= 0x10
    ss2 = eng.decaps(sk, ct)
    ss3 = eng.decaps(sk, _dev(bad))
    pk, sk, ss, ss2, ss3 = map(_host, (pk, sk, ss, ss2, ss3))
    opk, osk = orc.batch_keypair(alg, kc, 8)
    assert np.array_equal(pk, opk) and np.array_equal(sk, osk)
    oct_, oss = orc.batch_encaps(alg, opk, ec, 8)
    assert np.array_equal(ct_h, oct_) and np.array_equal(ss, oss) and np.array_equal(ss2, oss)
    assert np.array_equal(ss3, orc.batch_decaps(alg, osk, bad, 8))
