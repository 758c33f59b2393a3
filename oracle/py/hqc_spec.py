"""HQC (round-4 submission, version 2023-04-30) in pure Python.

TEST INFRASTRUCTURE ONLY -- imported by ``tests/`` and ``tests/golden`` only.

The reference selects HQC at ``quantum_resistant_p2p/crypto/key_exchange.py:189-309``
(variant map ``:206-223``: level 1/3/5 -> "HQC-128"/"HQC-192"/"HQC-256") and reaches
liboqs's HQC through ``quantum_resistant_p2p/vendor/oqs.py:318,348,372``.  liboqs
(0.12, which vendors the 2023-04-30 HQC reference implementation through PQClean) is
absent here and the reference holds no HQC vectors, so this restates that version's
published algorithm.  PARITY UNPINNED: no known-answer test pins it.
What is pinned: the sizes liboqs reports (pk/sk/ct/ss), and the Reed-Solomon generator
polynomial of HQC-128, recomputed here from the field and checked against the spec's
published coefficient list (tests/test_hqc_oracle.py).

Conventions restated (spec section 2 + the reference code's byte layout):

* vectors of F2[X]/(X^n - 1) are little-endian bit strings (bit i of byte i//8 = X^i);
* seedexpander(seed) = SHAKE256(seed || 0x02) squeezed in 8-byte units (a request of
  L bytes consumes ceil(L/8)*8 stream bytes);
* fixed-weight vectors (weight w): 4w stream bytes -> w LE32 r_i, support
  s_i = i + floor(r_i (n - i) / 2^32), then for i = w-2 .. 0: s_i := i if s_i equals
  some s_j, j > i (constant-weight sampling without rejection);
* random vector h: ceil(n/8) stream bytes, bits >= n cleared;
* KeyGen coins = sk_seed(40) || sigma(k) || pk_seed(40); x, y from seedexpander(sk_seed),
  h from seedexpander(pk_seed); s = x + y h; pk = pk_seed || s; sk = sk_seed || sigma || pk;
* Encaps coins = m(k) || salt(16); theta = SHAKE256(m || pk[0:80] || salt || 0x03)[0:64];
  r1, r2, e from seedexpander(theta[0:40]); u = r1 + r2 h;
  v = trunc_{n1 n2}(C.encode(m) + s r2 + e); ss = SHAKE256(m || u || v || 0x05)[0:64];
  ct = u || v || salt;
* Decaps: m' = C.decode(v - u y); re-encrypt with theta' = G(m' || pk[0:80] || salt);
  ss = K(m' or sigma || u || v) with the received u, v; the call returns -1 (OQS_ERROR)
  when the re-encryption differs (the reference's ``decap_secret`` then raises
  ``RuntimeError("Can not decapsulate secret")``, oqs.py:372-380);
* C = concatenated code: shortened Reed-Solomon [n1, k] over GF(2^8) (x^8+x^4+x^3+x^2+1,
  systematic, parity in symbols 0..2delta-1, message in 2delta..n1-1) inside a
  duplicated Reed-Muller RM(1,7) (symbol b -> 128 bits, bit j = b7 ^ <b0..6, j>,
  repeated `mult` times); RM decoding is the fast Hadamard transform of the summed copies
  with the first maximum |value| (sign -> bit 7), RS decoding any bounded-distance decoder
  (unique result for <= delta symbol errors).

Products with an operand read from a pk or ct (s, u) follow the reference's reduction
exactly: the linear product a is folded once, (a ^ (a >> n)) mod X^n, so stray bits a
malformed input carries above X^(n-1) are treated as the reference treats them.
"""
from __future__ import annotations

import hashlib

SEED_BYTES = 40
SALT_BYTES = 16
SS_BYTES = 64
D_SEEDEXP, D_G, D_K = 2, 3, 5

# n, n1, n2, w, w_r, w_e, k (message bytes), delta, RM multiplicity
_P = {
    "HQC-128": (17669, 46, 384, 66, 75, 75, 16, 15, 3),
    "HQC-192": (35851, 56, 640, 100, 114, 114, 24, 16, 5),
    "HQC-256": (57637, 90, 640, 131, 149, 149, 32, 29, 5),
}


def params(alg: str) -> dict:
    n, n1, n2, w, wr, we, k, delta, mult = _P[alg]
    nb = (n + 7) // 8
    n1n2 = n1 * n2
    return dict(n=n, n1=n1, n2=n2, n1n2=n1n2, w=w, wr=wr, we=we, k=k, delta=delta, mult=mult,
                nb=nb, vb=n1n2 // 8, pk=SEED_BYTES + nb, sk=SEED_BYTES + k + SEED_BYTES + nb,
                ct=nb + n1n2 // 8 + SALT_BYTES, ss=SS_BYTES,
                kp_coins=2 * SEED_BYTES + k, enc_coins=k + SALT_BYTES)


def sizes(alg: str) -> dict:
    p = params(alg)
    return {key: p[key] for key in ("pk", "sk", "ct", "ss", "kp_coins", "enc_coins")}


# ---------------------------------------------------------------- GF(2^8), poly 0x11D
GF_POLY = 0x11D
EXP = [0] * 512
LOG = [0] * 256
_x = 1
for _i in range(255):
    EXP[_i] = _x
    LOG[_x] = _i
    _x <<= 1
    if _x & 0x100:
        _x ^= GF_POLY
for _i in range(255, 512):
    EXP[_i] = EXP[_i - 255]


def gf_mul(a: int, b: int) -> int:
    if a == 0 or b == 0:
        return 0
    return EXP[LOG[a] + LOG[b]]


def gf_inv(a: int) -> int:
    return EXP[255 - LOG[a]]


def rs_generator(delta: int) -> list[int]:
    """g(x) = prod_{i=1}^{2 delta} (x - alpha^i), coefficients low -> high (monic)."""
    g = [1]
    for i in range(1, 2 * delta + 1):
        a = EXP[i]
        ng = [0] * (len(g) + 1)
        for j, c in enumerate(g):
            ng[j] ^= gf_mul(c, a)
            ng[j + 1] ^= c
        g = ng
    return g


# ---------------------------------------------------------------- SHAKE helpers
class SeedExpander:
    """SHAKE256(seed || 0x02), squeezed in 8-byte units."""

    def __init__(self, seed: bytes):
        self.h = hashlib.shake_256(bytes(seed) + bytes([D_SEEDEXP]))
        self.pos = 0

    def read(self, n: int) -> bytes:
        take = (n + 7) // 8 * 8
        out = self.h.digest(self.pos + take)[self.pos:self.pos + n]
        self.pos += take
        return out


def shake_ds(data: bytes, domain: int) -> bytes:
    return hashlib.shake_256(bytes(data) + bytes([domain])).digest(SS_BYTES)


def fixed_weight_support(se: SeedExpander, n: int, weight: int) -> list[int]:
    raw = se.read(4 * weight)
    r = [int.from_bytes(raw[4 * i:4 * i + 4], "little") for i in range(weight)]
    return remove_duplicates([i + ((r[i] * (n - i)) >> 32) for i in range(weight)])


def remove_duplicates(s: list[int]) -> list[int]:
    """The spec's serial duplicate removal (vect_set_random_fixed_weight, 2023-04-30):
    for i = w-2 .. 0, s_i := i when s_i equals some s_j with j > i."""
    s = list(s)
    weight = len(s)
    for i in range(weight - 2, -1, -1):
        if any(s[j] == s[i] for j in range(i + 1, weight)):
            s[i] = i
    return s


def support_to_int(sup: list[int]) -> int:
    v = 0
    for q in sup:
        v |= 1 << q
    return v


def random_vector(se: SeedExpander, n: int) -> int:
    nb = (n + 7) // 8
    return int.from_bytes(se.read(nb), "little") & ((1 << n) - 1)


def mul_sparse(sup: list[int], b: int, n: int) -> int:
    """sum_{q in sup} X^q b, reduced as the reference's vect_mul: fold the linear product once."""
    a = 0
    for q in sup:
        a ^= b << q
    return (a ^ (a >> n)) & ((1 << n) - 1)


# ---------------------------------------------------------------- concatenated code
def rs_encode(p: dict, msg: bytes) -> list[int]:
    n1, k = p["n1"], p["k"]
    g = rs_generator(p["delta"])
    par = n1 - k
    cdw = [0] * n1
    for i in range(k):
        gate = msg[k - 1 - i] ^ cdw[par - 1]
        tmp = [gf_mul(gate, c) for c in g]
        for j in range(par - 1, 0, -1):
            cdw[j] = cdw[j - 1] ^ tmp[j]
        cdw[0] = tmp[0]
    cdw[par:] = list(msg)
    return cdw


def rm_codeword(b: int) -> int:
    """RM(1,7): bit j of the 128-bit word = b7 ^ parity(b & 0x7F & j)."""
    out = 0
    for j in range(128):
        bit = ((b >> 7) ^ bin(b & j & 0x7F).count("1")) & 1
        out |= bit << j
    return out


def code_encode(p: dict, msg: bytes) -> int:
    mult = p["mult"]
    v = 0
    for i, sym in enumerate(rs_encode(p, msg)):
        cw = rm_codeword(sym)
        for c in range(mult):
            v |= cw << (128 * (i * mult + c))
    return v


def rm_decode_symbol(bits: int, mult: int) -> int:
    cnt = [0] * 128
    for c in range(mult):
        word = bits >> (128 * c)
        for j in range(128):
            cnt[j] += (word >> j) & 1
    t = cnt[:]
    h = 1
    while h < 128:  # Walsh-Hadamard, natural order: T[i] = sum_j (-1)^<i,j> cnt[j]
        for i0 in range(0, 128, 2 * h):
            for i in range(i0, i0 + h):
                a, b = t[i], t[i + h]
                t[i], t[i + h] = a + b, a - b
        h *= 2
    t[0] -= 64 * mult
    best_abs, best_val, best_pos = 0, 0, 0
    for i in range(128):
        a = abs(t[i])
        if a > best_abs:
            best_abs, best_val, best_pos = a, t[i], i
    return best_pos | (128 if best_val > 0 else 0)


def rs_syndromes(p: dict, r: list[int]) -> list[int]:
    return [_eval(r, EXP[i]) for i in range(1, 2 * p["delta"] + 1)]


def _eval(poly: list[int], x: int) -> int:
    acc = 0
    for c in reversed(poly):
        acc = gf_mul(acc, x) ^ c
    return acc


def rs_decode(p: dict, r: list[int]) -> list[int]:
    """Berlekamp-Massey + Chien + Forney over the n1 positions (bounded distance)."""
    n1, t2 = p["n1"], 2 * p["delta"]
    S = rs_syndromes(p, r)
    C, B, L, m, b = [1] + [0] * t2, [1] + [0] * t2, 0, 1, 1
    for i in range(t2):
        d = S[i]
        for j in range(1, L + 1):
            d ^= gf_mul(C[j], S[i - j])
        if d == 0:
            m += 1
            continue
        coef = gf_mul(d, gf_inv(b))
        T = C[:]
        for j in range(t2 + 1 - m):
            C[j + m] ^= gf_mul(coef, B[j])
        if 2 * L <= i:
            L, B, b, m = i + 1 - L, T, d, 1
        else:
            m += 1
    omega = [0] * t2  # S(x) C(x) mod x^(2 delta), S(x) = sum S_{i+1} x^i
    for i in range(t2):
        for j in range(i + 1):
            omega[i] ^= gf_mul(S[i - j], C[j])
    deriv = [C[j] if j % 2 == 1 else 0 for j in range(1, t2 + 1)]  # C'(x) coefficients
    out = list(r)
    for pos in range(n1):
        xinv = EXP[(255 - pos) % 255]
        if _eval(C, xinv) == 0:
            den = _eval(deriv, xinv)
            if den:
                out[pos] ^= gf_mul(_eval(omega, xinv), gf_inv(den))
    return out


def code_decode(p: dict, v: int) -> bytes:
    mult, n1 = p["mult"], p["n1"]
    span = 128 * mult
    r = [rm_decode_symbol((v >> (span * i)) & ((1 << span) - 1), mult) for i in range(n1)]
    c = rs_decode(p, r)
    return bytes(c[n1 - p["k"]:])


# ---------------------------------------------------------------- PKE / KEM
def _h_from_pk(p: dict, pk: bytes) -> int:
    return random_vector(SeedExpander(pk[:SEED_BYTES]), p["n"])


def _s_from_pk(p: dict, pk: bytes) -> int:
    return int.from_bytes(pk[SEED_BYTES:SEED_BYTES + p["nb"]], "little")  # unmasked, as loaded


def pke_encrypt(p: dict, m: bytes, theta: bytes, pk: bytes) -> tuple[int, int]:
    n = p["n"]
    se = SeedExpander(theta[:SEED_BYTES])
    h, s = _h_from_pk(p, pk), _s_from_pk(p, pk)
    r1 = fixed_weight_support(se, n, p["wr"])
    r2 = fixed_weight_support(se, n, p["wr"])
    e = fixed_weight_support(se, n, p["we"])
    u = support_to_int(r1) ^ mul_sparse(r2, h, n)
    v = code_encode(p, m) ^ mul_sparse(r2, s, n) ^ support_to_int(e)
    return u, v & ((1 << p["n1n2"]) - 1)


def keypair(alg: str, coins: bytes) -> tuple[bytes, bytes]:
    p = params(alg)
    n, k = p["n"], p["k"]
    sk_seed, sigma, pk_seed = coins[:SEED_BYTES], coins[SEED_BYTES:SEED_BYTES + k], \
        coins[SEED_BYTES + k:2 * SEED_BYTES + k]
    se = SeedExpander(sk_seed)
    x = fixed_weight_support(se, n, p["w"])
    y = fixed_weight_support(se, n, p["w"])
    h = random_vector(SeedExpander(pk_seed), n)
    s = support_to_int(x) ^ mul_sparse(y, h, n)
    pk = bytes(pk_seed) + s.to_bytes(p["nb"], "little")
    return pk, bytes(sk_seed) + bytes(sigma) + pk


def _theta(p: dict, m: bytes, pk: bytes, salt: bytes) -> bytes:
    return shake_ds(bytes(m) + bytes(pk[:2 * SEED_BYTES]) + bytes(salt), D_G)


def encaps(alg: str, pk: bytes, coins: bytes) -> tuple[bytes, bytes]:
    p = params(alg)
    m, salt = coins[:p["k"]], coins[p["k"]:p["k"] + SALT_BYTES]
    u, v = pke_encrypt(p, m, _theta(p, m, pk, salt), pk)
    ub, vb = u.to_bytes(p["nb"], "little"), v.to_bytes(p["vb"], "little")
    return ub + vb + bytes(salt), shake_ds(bytes(m) + ub + vb, D_K)


def decaps(alg: str, sk: bytes, ct: bytes) -> tuple[bytes, int]:
    """(ss, rc): rc = 0 on success, -1 when the re-encryption differs (ss still written)."""
    p = params(alg)
    n, k, nb, vb = p["n"], p["k"], p["nb"], p["vb"]
    sk_seed, sigma, pk = sk[:SEED_BYTES], sk[SEED_BYTES:SEED_BYTES + k], sk[SEED_BYTES + k:]
    ub, vbytes, salt = ct[:nb], ct[nb:nb + vb], ct[nb + vb:nb + vb + SALT_BYTES]
    se = SeedExpander(sk_seed)
    fixed_weight_support(se, n, p["w"])  # x (consumed, unused by decryption)
    y = fixed_weight_support(se, n, p["w"])
    u = int.from_bytes(ub, "little")
    v = int.from_bytes(vbytes, "little")
    m1 = code_decode(p, (v ^ mul_sparse(y, u, n)) & ((1 << p["n1n2"]) - 1))
    u2, v2 = pke_encrypt(p, m1, _theta(p, m1, pk, salt), pk)
    ok = u2.to_bytes(nb, "little") == bytes(ub) and v2.to_bytes(vb, "little") == bytes(vbytes)
    mc = m1 if ok else bytes(sigma)
    return shake_ds(mc + bytes(ub) + bytes(vbytes), D_K), (0 if ok else -1)
