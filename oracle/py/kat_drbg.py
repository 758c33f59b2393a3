"""NIST PQC known-answer-test DRBG (AES-256 CTR_DRBG) -- TEST INFRASTRUCTURE ONLY.

Restates ``randombytes_init`` / ``randombytes`` of the NIST PQC submission
package ``rng.c`` (the generator liboqs exposes as
``OQS_randombytes_nist_kat_init_256bit``).  The reference wrapper never calls
that switch (``quantum_resistant_p2p/vendor/oqs.py`` binds only
OQS_KEM_keypair/encaps/decaps, ``:318,348,372``), so KAT reproducibility in
this build goes through explicit coins: the DRBG output is chopped exactly as
liboqs's KEM code would consume it (one call per ``randombytes``), and handed
to the derandomised entry points.

AES-256 is implemented here from FIPS 197 (S-box derived from GF(2^8)
inversion, not a pasted table) so that no third-party crypto package is
needed.  Pure Python -- use for small counts only.
"""
from __future__ import annotations


def _xtime(a: int) -> int:
    a <<= 1
    if a & 0x100:
        a ^= 0x11B
    return a & 0xFF


def _gmul(a: int, b: int) -> int:
    r = 0
    while b:
        if b & 1:
            r ^= a
        a = _xtime(a)
        b >>= 1
    return r


def _make_sbox() -> list[int]:
    inv = [0] * 256
    for x in range(1, 256):
        for y in range(1, 256):
            if _gmul(x, y) == 1:
                inv[x] = y
                break
    sbox = []
    for x in range(256):
        b = inv[x]
        s = b
        for sh in range(1, 5):
            s ^= ((b << sh) | (b >> (8 - sh))) & 0xFF
        sbox.append(s ^ 0x63)
    return sbox


SBOX = _make_sbox()
_MUL2 = [_gmul(x, 2) for x in range(256)]
_MUL3 = [_gmul(x, 3) for x in range(256)]


def _expand_key(key: bytes) -> list[list[int]]:
    nk = len(key) // 4
    nr = nk + 6
    w = [list(key[4 * i:4 * i + 4]) for i in range(nk)]
    rcon = 1
    for i in range(nk, 4 * (nr + 1)):
        t = list(w[i - 1])
        if i % nk == 0:
            t = t[1:] + t[:1]
            t = [SBOX[b] for b in t]
            t[0] ^= rcon
            rcon = _xtime(rcon)
        elif nk > 6 and i % nk == 4:
            t = [SBOX[b] for b in t]
        w.append([a ^ b for a, b in zip(w[i - nk], t)])
    return [sum(w[4 * r:4 * r + 4], []) for r in range(nr + 1)]


def aes_encrypt_block(key: bytes, block: bytes, _cache: dict = {}) -> bytes:
    rk = _cache.get(key)
    if rk is None:
        rk = _expand_key(key)
        if len(_cache) > 64:
            _cache.clear()
        _cache[key] = rk
    s = [b ^ k for b, k in zip(block, rk[0])]
    nr = len(rk) - 1
    for r in range(1, nr + 1):
        s = [SBOX[b] for b in s]
        # ShiftRows: state is column-major, s[c*4 + row]
        s = [s[((c + row) % 4) * 4 + row] for c in range(4) for row in range(4)]
        if r != nr:
            t = []
            for c in range(4):
                a0, a1, a2, a3 = s[4 * c:4 * c + 4]
                t += [
                    _MUL2[a0] ^ _MUL3[a1] ^ a2 ^ a3,
                    a0 ^ _MUL2[a1] ^ _MUL3[a2] ^ a3,
                    a0 ^ a1 ^ _MUL2[a2] ^ _MUL3[a3],
                    _MUL3[a0] ^ a1 ^ a2 ^ _MUL2[a3],
                ]
            s = t
        s = [b ^ k for b, k in zip(s, rk[r])]
    return bytes(s)


class KatDrbg:
    """AES-256 CTR_DRBG, no derivation function, as in NIST PQC rng.c."""

    def __init__(self, entropy_input: bytes, personalization: bytes | None = None):
        assert len(entropy_input) == 48
        seed = bytearray(entropy_input)
        if personalization is not None:
            assert len(personalization) == 48
            seed = bytearray(a ^ b for a, b in zip(seed, personalization))
        self.key = bytes(32)
        self.v = bytearray(16)
        self._update(bytes(seed))
        self.reseed_counter = 1

    def _inc_v(self) -> None:
        for j in range(15, -1, -1):
            if self.v[j] == 0xFF:
                self.v[j] = 0
            else:
                self.v[j] += 1
                break

    def _update(self, provided: bytes | None) -> None:
        temp = bytearray()
        for _ in range(3):
            self._inc_v()
            temp += aes_encrypt_block(self.key, bytes(self.v))
        if provided is not None:
            temp = bytearray(a ^ b for a, b in zip(temp, provided))
        self.key = bytes(temp[:32])
        self.v = bytearray(temp[32:48])

    def randombytes(self, n: int) -> bytes:
        out = bytearray()
        while len(out) < n:
            self._inc_v()
            blk = aes_encrypt_block(self.key, bytes(self.v))
            out += blk[: min(16, n - len(out))]
        self._update(None)
        self.reseed_counter += 1
        return bytes(out)


def kat_seeds(count: int) -> list[bytes]:
    """The per-record 48-byte seeds of PQCgenKAT_kem (entropy = 0x00..0x2F)."""
    d = KatDrbg(bytes(range(48)))
    return [d.randombytes(48) for _ in range(count)]
