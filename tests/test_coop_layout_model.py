"""CPU model of the wave-cooperative Keccak-f[1600] data movement (csrc/keccak_coop.cuh).

The kernel spreads one sponge state over a wave: row y of the state in lanes 8y .. 8y + 7 (slot s
holds column (s + 4) mod 5, slots 0 / 6 / 7 replicate columns 4 / 0 / 1), and lanes 40-63 hold three
mirrors of row 4 so the column parity needs no mask.  This test replays `coop_init` and
`keccak_f_coop` lane by lane with the documented semantics of the cross-lane operations they use
(DPP row_ror / row_shr / row_shl with bound_ctrl and row_mask, v_permlane16_swap,
v_permlane32_swap, ds_bpermute) and checks the result against hashlib's SHA3 / SHAKE, so a change to
the layout, the masks or the replica bookkeeping can be checked without a GPU.  The GPU tests check
the kernels themselves (every single-shot ML-KEM / FrodoKEM / HQC test runs this permutation).
"""
import hashlib

import numpy as np

LANES = np.arange(64)
RHO = [0, 1, 62, 28, 27, 36, 44, 6, 55, 20, 3, 10, 43, 25, 39, 41, 45, 15, 21, 8, 18, 2, 61, 56, 14]
RC = [0x0000000000000001, 0x0000000000008082, 0x800000000000808A, 0x8000000080008000,
      0x000000000000808B, 0x0000000080000001, 0x8000000080008081, 0x8000000000008009,
      0x000000000000008A, 0x0000000000000088, 0x0000000080008009, 0x000000008000000A,
      0x000000008000808B, 0x800000000000008B, 0x8000000000008089, 0x8000000000008003,
      0x8000000000008002, 0x8000000000000080, 0x000000000000800A, 0x800000008000000A,
      0x8000000080008081, 0x8000000000008080, 0x0000000080000001, 0x8000000080008008]
M32 = 0xFFFFFFFF


# ---- cross-lane primitives (16-lane DPP rows, wave64)
def dpp(v, ctrl, row_mask=0xF, old=None):
    """DPP move with bound_ctrl: lanes whose source is outside the row read 0; rows whose
    row_mask bit is clear keep `old` (update_dpp) -- the kernel passes 0."""
    pos = LANES & 15
    kind, n = ctrl
    if kind == "shr":
        src, ok = LANES - n, pos >= n
    elif kind == "shl":
        src, ok = LANES + n, pos + n < 16
    else:  # "ror": lane l <- lane (l + n) mod 16 of its row
        src, ok = (LANES & ~15) | ((pos + n) & 15), np.ones(64, bool)
    out = np.where(ok, v[np.clip(src, 0, 63)], 0).astype(np.uint64)
    enabled = ((row_mask >> (LANES >> 4)) & 1).astype(bool)
    keep = np.zeros(64, np.uint64) if old is None else old
    return np.where(enabled, out, keep)


def permlane16_swap(a, b):
    """swap the odd 16-lane rows of a with the even rows of b"""
    a2, b2 = a.copy(), b.copy()
    for r in (0, 2):
        lo, hi = slice(16 * r, 16 * r + 16), slice(16 * r + 16, 16 * r + 32)
        a2[hi], b2[lo] = b[lo], a[hi]
    return a2, b2


def permlane32_swap(a, b):
    """swap the upper half of a with the lower half of b"""
    a2, b2 = a.copy(), b.copy()
    a2[32:], b2[:32] = b[:32], a[32:]
    return a2, b2


def bperm(addr, v):
    return v[(addr >> 2) & 63]


def alignbit(a, b, s):
    return ((((a << 32) | b) >> s) & M32).astype(np.uint64)


# ---- coop_init
def coop_init():
    sl = LANES & 7
    y = np.minimum(LANES >> 3, 4)  # lanes 40-63: three mirrors of row 4
    x = (sl + 4) % 5
    idx = x + 5 * y
    lane_xy = lambda xx, yy: 4 * (xx + 1 + 8 * yy)  # noqa: E731
    g0 = lane_xy((3 * y + x) % 5, x)
    r = np.array([RHO[i] for i in idx])
    n = r & 31
    return dict(
        idx=idx, g0=g0.astype(np.int64),
        m0=np.where((sl == 1) & (y == 0), M32, 0).astype(np.uint64),
        hi_slots=sl >= 6,
        shift=((32 - n) & 31).astype(np.uint64),
        swap=(r >= 32) != (n == 0),
    )


def coop_lane_of(i):
    return (i % 5) + 1 + 8 * (i // 5)


# ---- keccak_f_coop, statement by statement
def keccak_f_coop(lo, hi, c):
    sl_, sh_ = lo.copy(), hi.copy()
    for r in range(24):
        cl = sl_ ^ dpp(sl_, ("ror", 8), row_mask=0xB)
        ch = sh_ ^ dpp(sh_, ("ror", 8), row_mask=0xB)
        p0, p1 = permlane16_swap(cl, ch)
        t, t2 = p0 ^ p1, p0 ^ p1
        q0, q1 = permlane32_swap(t, t2)
        u, u2 = q0 ^ q1, q0 ^ q1
        cl, ch = permlane16_swap(u, u2)
        ml, mh = dpp(cl, ("shr", 1)), dpp(ch, ("shr", 1))
        pl, ph = dpp(cl, ("shl", 1)), dpp(ch, ("shl", 1))
        lo = lo ^ ml ^ alignbit(pl, ph, 31)
        hi = hi ^ mh ^ alignbit(ph, pl, 31)
        s_l = np.where(c["swap"], hi, lo)
        s_h = np.where(c["swap"], lo, hi)
        lo = alignbit(s_l, s_h, c["shift"])
        hi = alignbit(s_h, s_l, c["shift"])
        b0l, b0h = bperm(c["g0"], lo), bperm(c["g0"], hi)
        b1l, b1h = dpp(b0l, ("shl", 1)), dpp(b0h, ("shl", 1))
        b2l, b2h = dpp(b0l, ("shl", 2)), dpp(b0h, ("shl", 2))
        lo = (b0l ^ (~b1l & M32 & b2l)) ^ (RC[r] & M32 & c["m0"])
        hi = (b0h ^ (~b1h & M32 & b2h)) ^ ((RC[r] >> 32) & c["m0"])
        rl, rh = dpp(lo, ("shr", 5)), dpp(hi, ("shr", 5))
        sl_ = np.where(c["hi_slots"], rl, lo)
        sh_ = np.where(c["hi_slots"], rh, hi)
        lo, hi = sl_.copy(), sh_.copy()
    return lo, hi


def words_to_lanes(words, c):
    w = np.array([words[i] for i in c["idx"]], dtype=np.uint64)
    return w & M32, w >> 32


def lanes_to_words(lo, hi):
    return [int(lo[coop_lane_of(i)]) | (int(hi[coop_lane_of(i)]) << 32) for i in range(25)]


def check_replicas(lo, hi, c):
    """every lane holds the word its idx names (replicas and row-4 mirrors included)"""
    words = lanes_to_words(lo, hi)
    exp_lo, exp_hi = words_to_lanes(words, c)
    return np.array_equal(lo, exp_lo) and np.array_equal(hi, exp_hi)


def sponge(msg: bytes, rate: int, ds: int, out_len: int) -> bytes:
    c = coop_init()
    state = [0] * 25
    lo, hi = words_to_lanes(state, c)
    padded = bytearray(msg) + bytes([ds]) + bytes((-len(msg) - 1) % rate)
    padded[-1] |= 0x80
    for off in range(0, len(padded), rate):
        words = lanes_to_words(lo, hi)
        for i in range(rate // 8):
            words[i] ^= int.from_bytes(padded[off + 8 * i: off + 8 * i + 8], "little")
        lo, hi = words_to_lanes(words, c)
        lo, hi = keccak_f_coop(lo, hi, c)
        assert check_replicas(lo, hi, c)
    out = bytearray()
    while True:
        words = lanes_to_words(lo, hi)
        out += b"".join(w.to_bytes(8, "little") for w in words[: rate // 8])
        if len(out) >= out_len:
            return bytes(out[:out_len])
        lo, hi = keccak_f_coop(lo, hi, c)
        assert check_replicas(lo, hi, c)


def test_layout_lanes():
    c = coop_init()
    # every state word has exactly one canonical lane, and it names that word
    assert sorted(c["idx"][[coop_lane_of(i) for i in range(25)]].tolist()) == list(range(25))
    # lanes 32-63 all hold row 4, so the masked row_ror:8 step leaves 32-47 unpaired and cancels 48-63
    assert set((c["idx"][32:] // 5).tolist()) == {4}
    assert np.array_equal(c["idx"][48:56], c["idx"][56:64])


def test_sha3_256_one_block():
    msg = bytes(range(100))
    assert sponge(msg, 136, 0x06, 32) == hashlib.sha3_256(msg).digest()


def test_sha3_512_and_multiblock():
    msg = bytes((7 * i + 3) & 0xFF for i in range(300))  # three absorb blocks at rate 72... and more
    assert sponge(msg, 72, 0x06, 64) == hashlib.sha3_512(msg).digest()


def test_shake128_squeeze_three_blocks():
    msg = bytes(range(34))  # SampleNTT's rho || x || y shape
    assert sponge(msg, 168, 0x1F, 504) == hashlib.shake_128(msg).digest(504)
