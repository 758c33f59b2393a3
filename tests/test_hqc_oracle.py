"""HQC oracle checks (CPU) -- the C restatement (oracle/src/hqc.c) against the pure-Python
restatement (oracle/py/hqc_spec.py), the frozen vectors (tests/golden/hqc.json) and the
code's algebra.

PARITY UNPINNED against liboqs: no HQC known-answer vectors exist offline (DESIGN.md
section 2).  What the reference side pins: the sizes liboqs 0.12 reports for the
2023-04-30 HQC (test_sizes) and the HQC-128 Reed-Solomon generator polynomial published
with that version (test_rs_generator_hqc128), recomputed here from the field.
"""
import hashlib
import json
import random
from pathlib import Path

import pytest

import hqc_spec as H
import oracle as orc

GOLD = json.loads((Path(__file__).parent / "golden" / "hqc.json").read_text())
ALGS = ["HQC-128", "HQC-192", "HQC-256"]


def _sha(b: bytes) -> str:
    return hashlib.sha256(b).hexdigest()


def _tamper(ct: bytes, i: int) -> bytes:
    b = bytearray(ct)
    bit = (13 * i + 5) % (8 * len(b))
    b[bit // 8] ^= 1 << (bit % 8)
    return bytes(b)


@pytest.mark.parametrize("alg,sizes", [("HQC-128", (2249, 2305, 4433, 64)), ("HQC-192", (4522, 4586, 8978, 64)),
                                       ("HQC-256", (7245, 7317, 14421, 64))])
def test_sizes(alg, sizes):
    s = orc.sizes(alg)
    assert (s["pk"], s["sk"], s["ct"], s["ss"]) == sizes
    hs = H.sizes(alg)
    assert (hs["pk"], hs["sk"], hs["ct"], hs["ss"]) == sizes
    assert (hs["kp_coins"], hs["enc_coins"]) == (s["keypair_coins"], s["encaps_coins"])


def test_rs_generator_hqc128():
    # RS_POLY_COEFS of the 2023-04-30 HQC-128 parameter set (low -> high degree)
    published = [89, 69, 153, 116, 176, 117, 111, 75, 73, 233, 242, 233, 65, 210, 21, 139, 103, 173, 67, 118, 105,
                 210, 174, 110, 74, 69, 228, 82, 255, 181, 1]
    assert H.rs_generator(15) == published


@pytest.mark.parametrize("alg", ALGS)
def test_c_oracle_matches_golden(alg):
    for i, r in enumerate(GOLD[alg]["records"]):
        pk, sk = orc.keypair(alg, bytes.fromhex(r["kp_coins"]))
        assert _sha(pk) == r["pk"] and _sha(sk) == r["sk"] and pk[:64].hex() == r["pk64"]
        ct, ss = orc.encaps(alg, pk, bytes.fromhex(r["enc_coins"]))
        assert _sha(ct) == r["ct"] and ss.hex() == r["ss"] and ct[:64].hex() == r["ct64"]
        assert orc.decaps_rc(alg, sk, ct) == (ss, 0)
        tss, trc = orc.decaps_rc(alg, sk, _tamper(ct, i))
        assert tss.hex() == r["tampered_ss"] and trc == r["tampered_rc"] == -1


def test_python_spec_matches_golden():
    alg = "HQC-128"
    r = GOLD[alg]["records"][0]
    pk, sk = H.keypair(alg, bytes.fromhex(r["kp_coins"]))
    ct, ss = H.encaps(alg, pk, bytes.fromhex(r["enc_coins"]))
    assert _sha(pk) == r["pk"] and _sha(ct) == r["ct"] and ss.hex() == r["ss"]


@pytest.mark.parametrize("alg", ALGS)
def test_c_and_python_agree_random(alg):
    rng = random.Random(alg)
    s = H.sizes(alg)
    for _ in range(2):
        kc = rng.randbytes(s["kp_coins"])
        ec = rng.randbytes(s["enc_coins"])
        pk, sk = orc.keypair(alg, kc)
        assert (pk, sk) == H.keypair(alg, kc)
        ct, ss = orc.encaps(alg, pk, ec)
        assert (ct, ss) == H.encaps(alg, pk, ec)
        bad = bytearray(ct)
        bad[rng.randrange(len(bad))] ^= 1 << rng.randrange(8)
        assert orc.decaps_rc(alg, sk, bytes(bad)) == H.decaps(alg, sk, bytes(bad))


@pytest.mark.parametrize("alg", ALGS)
def test_stray_bits_above_n(alg):
    """Bits above X^(n-1) in a pk's s or a ct's u (malformed inputs) follow the reference's
    single-fold reduction; a ct carrying them is rejected (rc -1) with ss = K(sigma || ct)."""
    s = H.sizes(alg)
    p = H.params(alg)
    spare = 8 * p["nb"] - p["n"]
    assert spare > 0
    rng = random.Random(7)
    pk, sk = orc.keypair(alg, rng.randbytes(s["kp_coins"]))
    bad_pk = bytearray(pk)
    bad_pk[-1] |= 0x80  # highest spare bit of s
    ec = rng.randbytes(s["enc_coins"])
    got = orc.encaps(alg, bytes(bad_pk), ec)
    assert got == H.encaps(alg, bytes(bad_pk), ec)
    assert got != orc.encaps(alg, pk, ec)
    ct, ss = orc.encaps(alg, pk, ec)
    bad_ct = bytearray(ct)
    bad_ct[p["nb"] - 1] |= 0x80  # highest spare bit of u
    r = orc.decaps_rc(alg, sk, bytes(bad_ct))
    assert r == H.decaps(alg, sk, bytes(bad_ct)) and r[1] == -1


@pytest.mark.parametrize("alg", ALGS)
def test_rs_corrects_delta_errors(alg):
    p = H.params(alg)
    rng = random.Random(p["n"])
    for trial in range(4):
        msg = rng.randbytes(p["k"])
        c = H.rs_encode(p, msg)
        assert H.rs_syndromes(p, c) == [0] * (2 * p["delta"])
        r = list(c)
        for pos in rng.sample(range(p["n1"]), p["delta"] - trial):
            r[pos] ^= rng.randrange(1, 256)
        assert H.rs_decode(p, r) == c


@pytest.mark.parametrize("mult", [3, 5])
def test_rm_decodes_through_noise(mult):
    rng = random.Random(mult)
    for b in range(0, 256, 7):
        word = sum(H.rm_codeword(b) << (128 * c) for c in range(mult))
        for _ in range(20 * mult):  # well inside the duplicated RM(1,7) radius
            word ^= 1 << rng.randrange(128 * mult)
        assert H.rm_decode_symbol(word, mult) == b


@pytest.mark.parametrize("alg", ALGS)
def test_batch_driver_status(alg):
    """The threaded C batch driver reports each record's decaps return code."""
    import numpy as np
    s = orc.sizes(alg)
    n = 6
    kc = orc.bench_coins(n, s["keypair_coins"], seed=11)
    ec = orc.bench_coins(n, s["encaps_coins"], seed=12)
    pk, sk = orc.batch_keypair(alg, kc, 2)
    c, ss = orc.batch_encaps(alg, pk, ec, 2)
    c[1::2, 3] ^= 0x40
    ss2, st = orc.batch_decaps(alg, sk, c, 2, with_status=True)
    assert list(st) == [0, -1] * (n // 2)
    assert np.array_equal(ss2[0::2], ss[0::2]) and not np.array_equal(ss2[1::2], ss[1::2])
