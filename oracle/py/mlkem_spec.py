"""ML-KEM (FIPS 203) restated in plain Python -- TEST INFRASTRUCTURE ONLY.

This module is part of the parity oracle. It is imported only by ``tests/``,
``tests/golden/make_golden.py`` and never by the product path.

What it restates
----------------
The reference (ShadowCZEch/quantum-resistant-p2p) reaches ML-KEM only through
liboqs: ``quantum_resistant_p2p/vendor/oqs.py:318`` (OQS_KEM_keypair),
``:348`` (OQS_KEM_encaps) and ``:372`` (OQS_KEM_decaps), called from
``quantum_resistant_p2p/crypto/key_exchange.py:133,156,179``.  liboqs (pinned
only by the wrapper string "vendored-12.0.0", ``oqs.py:46``; struct layout of
liboqs 0.12.x, ``oqs.py:241-253``) is absent from the reference tree
(``.MISSING_LARGE_BLOBS:1``), so the arithmetic is restated from the published
algorithm: NIST FIPS 203 (Aug 2024), Algorithms 3-18, with the randomness
granularity of the pq-crystals "standard" code that liboqs 0.12 wraps
(KeyGen draws d||z in ONE 64-byte randombytes call, Encaps draws m in ONE
32-byte call).

Written directly from the FIPS 203 pseudo-code: canonical mod-q integers, no
Montgomery/Barrett tricks, so that it is an independent check of the C
restatement in ``oracle/src/mlkem.c`` and of the HIP kernels.
"""
from __future__ import annotations

import hashlib

Q = 3329
N = 256

# (k, eta1, eta2, du, dv) -- FIPS 203 Table 2
PARAMS = {
    "ML-KEM-512": (2, 3, 2, 10, 4),
    "ML-KEM-768": (3, 2, 2, 10, 4),
    "ML-KEM-1024": (4, 2, 2, 11, 5),
}


def sizes(alg: str) -> dict:
    k, _e1, _e2, du, dv = PARAMS[alg]
    return {
        "pk": 384 * k + 32,
        "sk": 768 * k + 96,
        "ct": 32 * (du * k + dv),
        "ss": 32,
        "keypair_coins": 64,
        "encaps_coins": 32,
    }


def _bitrev7(i: int) -> int:
    return int(format(i, "07b")[::-1], 2)


ZETAS = [pow(17, _bitrev7(i), Q) for i in range(128)]
GAMMAS = [pow(17, 2 * _bitrev7(i) + 1, Q) for i in range(128)]


# --- hash primitives (FIPS 203 section 4.1) --------------------------------
def H(s: bytes) -> bytes:
    return hashlib.sha3_256(s).digest()


def G(s: bytes) -> tuple[bytes, bytes]:
    d = hashlib.sha3_512(s).digest()
    return d[:32], d[32:]


def J(s: bytes) -> bytes:
    return hashlib.shake_256(s).digest(32)


def PRF(eta: int, s: bytes, b: int) -> bytes:
    return hashlib.shake_256(s + bytes([b])).digest(64 * eta)


# --- encodings (Algorithms 5, 6) --------------------------------------------
def byte_encode(d: int, F: list[int]) -> bytes:
    bits = 0
    acc = 0
    out = bytearray()
    for a in F:
        acc |= (a & ((1 << d) - 1)) << bits
        bits += d
        while bits >= 8:
            out.append(acc & 0xFF)
            acc >>= 8
            bits -= 8
    assert bits == 0
    return bytes(out)


def byte_decode(d: int, B: bytes) -> list[int]:
    m = Q if d == 12 else (1 << d)
    acc = int.from_bytes(B, "little")
    return [((acc >> (d * i)) & ((1 << d) - 1)) % m for i in range(N)]


def compress(d: int, x: int) -> int:
    # round(2^d / q * x) mod 2^d, ties impossible since q is odd
    return (((x << d) + Q // 2) // Q) & ((1 << d) - 1)


def decompress(d: int, y: int) -> int:
    return (Q * y + (1 << (d - 1))) >> d


# --- sampling (Algorithms 7, 8) --------------------------------------------
def sample_ntt(B: bytes) -> list[int]:
    assert len(B) == 34
    nbytes = 168 * 3
    while True:
        stream = hashlib.shake_128(B).digest(nbytes)
        a = []
        pos = 0
        while len(a) < N and pos + 3 <= len(stream):
            c0, c1, c2 = stream[pos], stream[pos + 1], stream[pos + 2]
            pos += 3
            d1 = c0 + 256 * (c1 % 16)
            d2 = c1 // 16 + 16 * c2
            if d1 < Q:
                a.append(d1)
            if d2 < Q and len(a) < N:
                a.append(d2)
        if len(a) == N:
            return a
        nbytes += 168


def sample_cbd(eta: int, B: bytes) -> list[int]:
    assert len(B) == 64 * eta
    bits = int.from_bytes(B, "little")
    f = []
    for i in range(N):
        x = sum((bits >> (2 * i * eta + j)) & 1 for j in range(eta))
        y = sum((bits >> (2 * i * eta + eta + j)) & 1 for j in range(eta))
        f.append((x - y) % Q)
    return f


# --- NTT (Algorithms 9-12) ---------------------------------------------------
def ntt(f: list[int]) -> list[int]:
    f = list(f)
    i = 1
    length = 128
    while length >= 2:
        for start in range(0, N, 2 * length):
            zeta = ZETAS[i]
            i += 1
            for j in range(start, start + length):
                t = zeta * f[j + length] % Q
                f[j + length] = (f[j] - t) % Q
                f[j] = (f[j] + t) % Q
        length //= 2
    return f


def ntt_inv(f: list[int]) -> list[int]:
    f = list(f)
    i = 127
    length = 2
    while length <= 128:
        for start in range(0, N, 2 * length):
            zeta = ZETAS[i]
            i -= 1
            for j in range(start, start + length):
                t = f[j]
                f[j] = (t + f[j + length]) % Q
                f[j + length] = zeta * (f[j + length] - t) % Q
        length *= 2
    return [x * 3303 % Q for x in f]


def multiply_ntts(f: list[int], g: list[int]) -> list[int]:
    h = [0] * N
    for i in range(128):
        a0, a1, b0, b1 = f[2 * i], f[2 * i + 1], g[2 * i], g[2 * i + 1]
        h[2 * i] = (a0 * b0 + a1 * b1 * GAMMAS[i]) % Q
        h[2 * i + 1] = (a0 * b1 + a1 * b0) % Q
    return h


def _add(a, b):
    return [(x + y) % Q for x, y in zip(a, b)]


def _sub(a, b):
    return [(x - y) % Q for x, y in zip(a, b)]


# --- K-PKE (Algorithms 13-15) -----------------------------------------------
def _matrix(rho: bytes, k: int):
    # A_hat[i][j] = SampleNTT(rho || j || i)
    return [[sample_ntt(rho + bytes([j, i])) for j in range(k)] for i in range(k)]


def kpke_keygen(alg: str, d: bytes):
    k, eta1, _eta2, _du, _dv = PARAMS[alg]
    rho, sigma = G(d + bytes([k]))
    A = _matrix(rho, k)
    nonce = 0
    s = []
    for _ in range(k):
        s.append(sample_cbd(eta1, PRF(eta1, sigma, nonce)))
        nonce += 1
    e = []
    for _ in range(k):
        e.append(sample_cbd(eta1, PRF(eta1, sigma, nonce)))
        nonce += 1
    s_hat = [ntt(p) for p in s]
    e_hat = [ntt(p) for p in e]
    t_hat = []
    for i in range(k):
        acc = [0] * N
        for j in range(k):
            acc = _add(acc, multiply_ntts(A[i][j], s_hat[j]))
        t_hat.append(_add(acc, e_hat[i]))
    ek = b"".join(byte_encode(12, p) for p in t_hat) + rho
    dk = b"".join(byte_encode(12, p) for p in s_hat)
    return ek, dk


def kpke_encrypt(alg: str, ek: bytes, m: bytes, r: bytes) -> bytes:
    k, eta1, eta2, du, dv = PARAMS[alg]
    t_hat = [byte_decode(12, ek[384 * i:384 * (i + 1)]) for i in range(k)]
    rho = ek[384 * k:384 * k + 32]
    A = _matrix(rho, k)
    nonce = 0
    y = []
    for _ in range(k):
        y.append(sample_cbd(eta1, PRF(eta1, r, nonce)))
        nonce += 1
    e1 = []
    for _ in range(k):
        e1.append(sample_cbd(eta2, PRF(eta2, r, nonce)))
        nonce += 1
    e2 = sample_cbd(eta2, PRF(eta2, r, nonce))
    y_hat = [ntt(p) for p in y]
    u = []
    for i in range(k):
        acc = [0] * N
        for j in range(k):
            acc = _add(acc, multiply_ntts(A[j][i], y_hat[j]))  # A^T
        u.append(_add(ntt_inv(acc), e1[i]))
    mu = [decompress(1, b) for b in byte_decode(1, m)]
    acc = [0] * N
    for j in range(k):
        acc = _add(acc, multiply_ntts(t_hat[j], y_hat[j]))
    v = _add(_add(ntt_inv(acc), e2), mu)
    c1 = b"".join(byte_encode(du, [compress(du, x) for x in p]) for p in u)
    c2 = byte_encode(dv, [compress(dv, x) for x in v])
    return c1 + c2


def kpke_decrypt(alg: str, dk: bytes, c: bytes) -> bytes:
    k, _eta1, _eta2, du, dv = PARAMS[alg]
    c1 = c[:32 * du * k]
    c2 = c[32 * du * k:]
    u = [[decompress(du, x) for x in byte_decode(du, c1[32 * du * i:32 * du * (i + 1)])]
         for i in range(k)]
    v = [decompress(dv, x) for x in byte_decode(dv, c2)]
    s_hat = [byte_decode(12, dk[384 * i:384 * (i + 1)]) for i in range(k)]
    acc = [0] * N
    for j in range(k):
        acc = _add(acc, multiply_ntts(s_hat[j], ntt(u[j])))
    w = _sub(v, ntt_inv(acc))
    return byte_encode(1, [compress(1, x) for x in w])


# --- ML-KEM internal (Algorithms 16-18) --------------------------------------
def keypair_derand(alg: str, coins: bytes) -> tuple[bytes, bytes]:
    """coins = d || z (64 bytes) -- one randombytes(64) call in liboqs/pq-crystals."""
    assert len(coins) == 64
    d, z = coins[:32], coins[32:]
    ek, dk_pke = kpke_keygen(alg, d)
    dk = dk_pke + ek + H(ek) + z
    return ek, dk


def ek_modulus_ok(alg: str, ek: bytes) -> bool:
    """FIPS 203 section 7.2 encapsulation-key check."""
    k = PARAMS[alg][0]
    for i in range(k):
        chunk = ek[384 * i:384 * (i + 1)]
        if byte_encode(12, byte_decode(12, chunk)) != chunk:
            return False
    return True


def encaps_derand(alg: str, ek: bytes, m: bytes) -> tuple[bytes, bytes]:
    """m = 32 coins (one randombytes(32) call). Returns (ct, ss)."""
    assert len(m) == 32
    K, r = G(m + H(ek))
    c = kpke_encrypt(alg, ek, m, r)
    return c, K


def decaps(alg: str, dk: bytes, c: bytes) -> bytes:
    k = PARAMS[alg][0]
    dk_pke = dk[:384 * k]
    ek = dk[384 * k:768 * k + 32]
    h = dk[768 * k + 32:768 * k + 64]
    z = dk[768 * k + 64:768 * k + 96]
    m2 = kpke_decrypt(alg, dk_pke, c)
    K2, r2 = G(m2 + h)
    Kbar = J(z + c)
    c2 = kpke_encrypt(alg, ek, m2, r2)
    return K2 if c2 == c else Kbar
