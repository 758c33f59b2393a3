"""FrodoKEM (round-3 specification, SHAKE and AES variants) in Python/numpy.

TEST INFRASTRUCTURE ONLY -- imported by ``tests/`` and ``tests/golden`` only.

The reference selects FrodoKEM at ``quantum_resistant_p2p/crypto/key_exchange.py:312-449``
(variant maps ``:332-343``) and reaches liboqs's FrodoKEM through
``quantum_resistant_p2p/vendor/oqs.py:318,348,372``.  liboqs is absent, so this
restates the FrodoKEM round-3 specification (2021-06-04, "FrodoKEM: Learning With
Errors Key Encapsulation", Algorithms 1-15 + section 2.2 parameter tables), with
the byte conventions of its reference code (the code liboqs 0.12 vendors):

* KeyGen draws s || seedSE || z (len_s + len_seedSE + 16 bytes) in one call;
  seedA = SHAKE(z, 16); (S^T || E) = sample(SHAKE(0x5F || seedSE)).
* Encaps draws mu (len_mu bytes); pkh = SHAKE(pk, len_pkh);
  (seedSE || k) = SHAKE(pkh || mu); (S' || E' || E'') = sample(SHAKE(0x96 || seedSE));
  ss = SHAKE(c1 || c2 || k).
* Decaps re-encrypts and selects k' or s with a constant-time compare.

SHAKE128 is the hash for FrodoKEM-640, SHAKE256 for -976/-1344; A is generated
row-wise with SHAKE128(LE16(i) || seedA) (SHAKE variants) or AES-128-ECB over
(LE16(i) || LE16(j) || 0...) blocks keyed by seedA (AES variants).
"""
from __future__ import annotations

import hashlib

import numpy as np

from kat_drbg import aes_encrypt_block

NBAR = 8

# n, logq, B (extracted bits), len_sec (CRYPTO_BYTES), CDF table
_BASE = {
    640: (640, 15, 2, 16, [4643, 13363, 20579, 25843, 29227, 31145, 32103, 32525,
                           32689, 32745, 32762, 32766, 32767]),
    976: (976, 16, 3, 24, [5638, 15915, 23689, 28571, 31116, 32217, 32613, 32731,
                           32760, 32766, 32767]),
    1344: (1344, 16, 4, 32, [9142, 23462, 30338, 32361, 32725, 32765, 32767]),
}

ALGS = [f"FrodoKEM-{n}-{prg}" for n in (640, 976, 1344) for prg in ("AES", "SHAKE")]


def params(alg: str) -> dict:
    _, n_s, prg = alg.split("-")
    n, logq, B, sec, cdf = _BASE[int(n_s)]
    p = {
        "n": n, "logq": logq, "B": B, "sec": sec, "cdf": cdf, "prg": prg,
        "len_seedA": 16, "len_mu": B * NBAR * NBAR // 8,
    }
    p["pk"] = 16 + logq * n * NBAR // 8
    p["ct"] = logq * n * NBAR // 8 + logq * NBAR * NBAR // 8
    p["sk"] = sec + p["pk"] + 2 * n * NBAR + sec
    p["ss"] = sec
    p["keypair_coins"] = 2 * sec + 16
    p["encaps_coins"] = p["len_mu"]
    return p


def sizes(alg: str) -> dict:
    p = params(alg)
    return {k: p[k] for k in ("pk", "sk", "ct", "ss", "keypair_coins", "encaps_coins")}


def _shake(p: dict, data: bytes, outlen: int) -> bytes:
    if p["n"] == 640:
        return hashlib.shake_128(data).digest(outlen)
    return hashlib.shake_256(data).digest(outlen)


def gen_a(p: dict, seed_a: bytes) -> np.ndarray:
    n = p["n"]
    A = np.zeros((n, n), dtype=np.uint16)
    if p["prg"] == "SHAKE":
        for i in range(n):
            row = hashlib.shake_128(i.to_bytes(2, "little") + seed_a).digest(2 * n)
            A[i] = np.frombuffer(row, dtype="<u2")
    else:
        for i in range(n):
            for j in range(0, n, 8):
                blk = i.to_bytes(2, "little") + j.to_bytes(2, "little") + bytes(12)
                A[i, j:j + 8] = np.frombuffer(aes_encrypt_block(seed_a, blk), dtype="<u2")
    return A


def sample(p: dict, r: np.ndarray) -> np.ndarray:
    """CDF sampler: r are 16-bit words; returns values mod 2^16 (two's complement)."""
    r = r.astype(np.int64)
    prnd = r >> 1
    sign = r & 1
    s = np.zeros_like(r)
    for c in p["cdf"][:-1]:
        s += ((c - prnd) < 0).astype(np.int64)
    out = np.where(sign == 1, -s, s)
    return (out & 0xFFFF).astype(np.uint16)


def pack(vals: np.ndarray, d: int) -> bytes:
    """MSB-first bit packing of d-bit values (frodo_pack)."""
    acc = 0
    for v in vals.astype(np.int64).ravel().tolist():
        acc = (acc << d) | (v & ((1 << d) - 1))
    nbits = d * vals.size
    return acc.to_bytes(nbits // 8, "big")


def unpack(data: bytes, count: int, d: int) -> np.ndarray:
    acc = int.from_bytes(data, "big")
    nbits = 8 * len(data)
    out = np.empty(count, dtype=np.uint16)
    mask = (1 << d) - 1
    for i in range(count):
        out[i] = (acc >> (nbits - d * (i + 1))) & mask
    return out


def encode(p: dict, mu: bytes) -> np.ndarray:
    B, logq = p["B"], p["logq"]
    bits = int.from_bytes(mu, "little")
    vals = [((bits >> (B * i)) & ((1 << B) - 1)) << (logq - B) for i in range(NBAR * NBAR)]
    return np.array(vals, dtype=np.uint16).reshape(NBAR, NBAR)


def decode(p: dict, M: np.ndarray) -> bytes:
    B, logq = p["B"], p["logq"]
    qmask = (1 << logq) - 1
    bits = 0
    for i, v in enumerate(M.astype(np.int64).ravel().tolist()):
        t = (((v & qmask) + (1 << (logq - B - 1))) >> (logq - B)) & ((1 << B) - 1)
        bits |= t << (B * i)
    return bits.to_bytes(p["len_mu"], "little")


def _mm(a: np.ndarray, b: np.ndarray) -> np.ndarray:
    return (a.astype(np.int64) @ b.astype(np.int64)) & 0xFFFF


def keypair_derand(alg: str, coins: bytes) -> tuple[bytes, bytes]:
    p = params(alg)
    n, sec, logq = p["n"], p["sec"], p["logq"]
    assert len(coins) == 2 * sec + 16
    s, seed_se, z = coins[:sec], coins[sec:2 * sec], coins[2 * sec:]
    seed_a = _shake(p, z, 16)
    r = np.frombuffer(_shake(p, b"\x5f" + seed_se, 4 * n * NBAR), dtype="<u2")
    St = sample(p, r[:n * NBAR]).reshape(NBAR, n)          # S^T, row-major nbar x n
    E = sample(p, r[n * NBAR:]).reshape(n, NBAR)
    A = gen_a(p, seed_a)
    Bm = (_mm(A, St.T) + E) & 0xFFFF
    pk = seed_a + pack(Bm & ((1 << logq) - 1), logq)
    pkh = _shake(p, pk, sec)
    sk = s + pk + St.astype("<u2").tobytes() + pkh
    return pk, sk


def _encrypt_core(p, pk, seed_se, mu):
    n, logq = p["n"], p["logq"]
    qmask = (1 << logq) - 1
    seed_a = pk[:16]
    r = np.frombuffer(_shake(p, b"\x96" + seed_se, (2 * n + NBAR) * NBAR * 2), dtype="<u2")
    Sp = sample(p, r[:n * NBAR]).reshape(NBAR, n)
    Ep = sample(p, r[n * NBAR:2 * n * NBAR]).reshape(NBAR, n)
    Epp = sample(p, r[2 * n * NBAR:]).reshape(NBAR, NBAR)
    A = gen_a(p, seed_a)
    Bp = (_mm(Sp, A) + Ep) & qmask
    Bpk = unpack(pk[16:], n * NBAR, logq).reshape(n, NBAR)
    V = (_mm(Sp, Bpk) + Epp) & qmask
    C = (V + encode(p, mu)) & qmask
    return Bp, C


def encaps_derand(alg: str, pk: bytes, mu: bytes) -> tuple[bytes, bytes]:
    p = params(alg)
    sec, logq = p["sec"], p["logq"]
    assert len(mu) == p["len_mu"]
    pkh = _shake(p, pk, sec)
    g = _shake(p, pkh + mu, 2 * sec)
    seed_se, k = g[:sec], g[sec:]
    Bp, C = _encrypt_core(p, pk, seed_se, mu)
    ct = pack(Bp, logq) + pack(C, logq)
    ss = _shake(p, ct + k, sec)
    return ct, ss


def decaps(alg: str, sk: bytes, ct: bytes) -> bytes:
    p = params(alg)
    n, sec, logq = p["n"], p["sec"], p["logq"]
    qmask = (1 << logq) - 1
    s = sk[:sec]
    pk = sk[sec:sec + p["pk"]]
    St = np.frombuffer(sk[sec + p["pk"]:sec + p["pk"] + 2 * n * NBAR], dtype="<u2").reshape(NBAR, n)
    pkh = sk[sec + p["pk"] + 2 * n * NBAR:]
    c1len = logq * n * NBAR // 8
    Bp = unpack(ct[:c1len], n * NBAR, logq).reshape(NBAR, n)
    C = unpack(ct[c1len:], NBAR * NBAR, logq).reshape(NBAR, NBAR)
    M = (C.astype(np.int64) - _mm(Bp, St.T)) & qmask
    mu2 = decode(p, M)
    g = _shake(p, pkh + mu2, 2 * sec)
    seed_se2, k2 = g[:sec], g[sec:]
    Bp2, C2 = _encrypt_core(p, pk, seed_se2, mu2)
    ok = np.array_equal(Bp2, Bp) and np.array_equal(C2, C)
    return _shake(p, ct + (k2 if ok else s), sec)
