"""CPU: pin the parity oracle before trusting it.

* Keccak / SHA3 / SHAKE of both restatements against Python hashlib;
* the NIST KAT DRBG against the per-record seeds published at the top of every
  NIST PQC KEM KAT file (count = 0 and 1) and AES against FIPS 197 Appendix C;
* the C oracle (oracle/liboracle.so) against the committed golden vectors
  (tests/golden, made by the independent pure-Python restatement), including
  every one of the 1024 ML-KEM-768 KAT-DRBG records (BASELINE.json configs[0]).

liboqs's own KAT digests are not available offline, so ML-KEM / FrodoKEM bytes are
pinned to the restatements, not to liboqs ("parity unpinned vs liboqs").
"""
import hashlib
import json
import os

import numpy as np
import pytest

import oracle as orc

NIST_SEED_0 = ("061550234D158C5EC95595FE04EF7A25767F2E24CC2BC479D09D86DC9ABCFDE7"
               "056A8C266F9EF97ED08541DBD2E1FFA1")
NIST_SEED_1 = ("D81C4D8D734FCBFBEADE3D3F8A039FAA2A2C9957E835AD55B22E75BF57BB556A"
               "C81ADDE6AEEB4A5A875C3BFCADFA958F")


@pytest.mark.parametrize("n", [0, 1, 7, 33, 71, 72, 73, 135, 136, 137, 167, 168, 169, 333, 1184])
def test_hashes_vs_hashlib(n):
    data = os.urandom(n)
    assert orc.hash_(0, data, 500) == hashlib.shake_128(data).digest(500)
    assert orc.hash_(1, data, 300) == hashlib.shake_256(data).digest(300)
    assert orc.hash_(2, data, 32) == hashlib.sha3_256(data).digest()
    assert orc.hash_(3, data, 64) == hashlib.sha3_512(data).digest()


def test_aes_fips197():
    pt = bytes.fromhex("00112233445566778899aabbccddeeff")
    assert orc.aes_block(bytes(range(16)), pt).hex() == "69c4e0d86a7b0430d8cdb78070b4c55a"
    assert orc.aes_block(bytes(range(32)), pt).hex() == "8ea2b7ca516745bfeafc49904b496089"
    import kat_drbg
    assert kat_drbg.aes_encrypt_block(bytes(range(16)), pt).hex() == "69c4e0d86a7b0430d8cdb78070b4c55a"


def test_kat_drbg_reproduces_nist_seeds():
    seeds, _, _ = orc.kat_coins(2, 64, 32)
    assert seeds[0].tobytes().hex().upper() == NIST_SEED_0
    assert seeds[1].tobytes().hex().upper() == NIST_SEED_1
    import kat_drbg
    py = kat_drbg.kat_seeds(2)
    assert py[0].hex().upper() == NIST_SEED_0 and py[1].hex().upper() == NIST_SEED_1


def _kat_check(golden, alg):
    g = golden[alg]
    n = g["count"]
    _, kc, ec = orc.kat_coins(n, g["kp_coins"], g["enc_coins"])
    pk, sk = orc.batch_keypair(alg, kc)
    ct, ss = orc.batch_encaps(alg, pk, ec)
    ss2 = orc.batch_decaps(alg, sk, ct)
    assert np.array_equal(ss, ss2)
    for name, arr in (("pk", pk), ("sk", sk), ("ct", ct), ("ss", ss)):
        assert hashlib.sha256(arr.tobytes()).hexdigest() == g["digests"][name], (alg, name)
    for r in g["records"]:
        i = r["count"]
        assert r["ss"] == ss[i].tobytes().hex()
        assert r["ct_sha256"] == hashlib.sha256(ct[i].tobytes()).hexdigest()
        assert r["pk_sha256"] == hashlib.sha256(pk[i].tobytes()).hexdigest()


@pytest.mark.parametrize("alg", ["ML-KEM-512", "ML-KEM-768", "ML-KEM-1024"])
def test_c_oracle_matches_golden_mlkem(golden_dir, alg):
    _kat_check(json.loads((golden_dir / "kat_mlkem.json").read_text()), alg)


@pytest.mark.parametrize("alg", ["FrodoKEM-640-SHAKE", "FrodoKEM-976-SHAKE", "FrodoKEM-1344-SHAKE",
                                 "FrodoKEM-640-AES", "FrodoKEM-976-AES", "FrodoKEM-1344-AES"])
def test_c_oracle_matches_golden_frodo(golden_dir, alg):
    _kat_check(json.loads((golden_dir / "kat_frodo.json").read_text()), alg)


def test_c_oracle_tampered(golden_dir):
    g = json.loads((golden_dir / "tampered.json").read_text())
    alg = g["alg"]
    pk, sk = orc.keypair(alg, bytes.fromhex(g["keypair_coins"]))
    ct, ss = orc.encaps(alg, pk, bytes.fromhex(g["encaps_coins"]))
    assert ss.hex() == g["ss_valid"]
    for case in g["cases"]:
        bad = bytearray(ct)
        bad[case["bit"] // 8] ^= 1 << (case["bit"] % 8)
        assert orc.decaps(alg, sk, bytes(bad)).hex() == case["ss"]


def test_bench_coins(golden_dir):
    g = json.loads((golden_dir / "coins.json").read_text())
    for it in g["items"]:
        got = orc.bench_coins(1, g["len"], g["seed"], it["i"])
        assert got[0].tobytes().hex() == it["coins"]


@pytest.mark.parametrize("alg", ["ML-KEM-512", "ML-KEM-768", "ML-KEM-1024"])
def test_c_vs_python_random(alg):
    import mlkem_spec as M
    for _ in range(3):
        kc, ec = os.urandom(64), os.urandom(32)
        pk, sk = orc.keypair(alg, kc)
        assert (pk, sk) == M.keypair_derand(alg, kc)
        c, ss = orc.encaps(alg, pk, ec)
        assert (c, ss) == M.encaps_derand(alg, pk, ec)
        bad = bytearray(c)
        bad[len(c) - 1] ^= 0x80
        assert orc.decaps(alg, sk, bytes(bad)) == M.decaps(alg, sk, bytes(bad))


def test_modulus_check_rejects_noncanonical():
    alg = "ML-KEM-768"
    pk, _ = orc.keypair(alg, bytes(64))
    bad = bytearray(pk)
    bad[0] = 0xFF
    bad[1] |= 0x0F
    with pytest.raises(RuntimeError):
        orc.encaps(alg, bytes(bad), bytes(32))
