"""HQC's duplicate removal as the HIP kernels run it (csrc/hqc.hip dedupe_wave: one wave per
vector, element 64e + l in lane l's register e, one v_readlane broadcast and one ballot per
register per step, masked to j > i), checked on the CPU against the spec's serial loop
(oracle/py/hqc_spec.py remove_duplicates, restating vect_set_random_fixed_weight of the
2023-04-30 HQC).  Also kept: the round-1 closed form (pointer jumping over the workgroup).

Serial loop: for i = w-2 .. 0, s_i := i when s_i equals some s_j with j > i.
Closed form: s_i is replaced iff (s_j == s_i for some j > i, original values) or
(i < s_i < w and s_{s_i} is replaced) -- resolved by pointer jumping in ceil(log2 w) rounds,
in place, in any update order within a round (the GPU's threads race within a round).

Inputs are crafted so collisions, index collisions and long chains are common (at real HQC
sizes they are rare, so random supports would not exercise the rule).
"""
import random

import pytest

import hqc_spec as H

NONE = None


def closed_form(s, order_rng=None):
    w = len(s)
    rep = [any(s[j] == s[i] for j in range(i + 1, w)) for i in range(w)]
    ptr = [s[i] if i < s[i] < w else NONE for i in range(w)]
    rounds = (w - 1).bit_length()
    assert 2 ** rounds >= w
    for _ in range(rounds):
        order = list(range(w))
        if order_rng is not None:  # in-place updates in an arbitrary order within the round
            order_rng.shuffle(order)
            for e in order:
                p = ptr[e]
                if p is not NONE:
                    rep[e] = rep[e] or rep[p]
                    ptr[e] = ptr[p]
        else:  # synchronous rounds
            nrep = [rep[e] or (ptr[e] is not NONE and rep[ptr[e]]) for e in range(w)]
            nptr = [ptr[ptr[e]] if ptr[e] is not NONE else NONE for e in range(w)]
            rep, ptr = nrep, nptr
    return [i if rep[i] else s[i] for i in range(w)]


def wave_form(s):
    """dedupe_wave restated: registers v[e][lane], ballots as 64-bit masks."""
    w = len(s)
    ne = (w + 63) // 64
    sentinel = 0xFFFFFFFF
    v = [[s[64 * e + l] if 64 * e + l < w else sentinel for l in range(64)] for e in range(ne)]
    for i in range(w - 2, -1, -1):
        ei, li = i >> 6, i & 63
        si = v[ei][li]  # v_readlane
        hit = 0
        for e in range(ne):
            if 64 * e + 63 <= i:
                continue
            m = sum(1 << l for l in range(64) if v[e][l] == si)  # ballot
            if 64 * e <= i:
                m &= (~0 << (i - 64 * e + 1)) & ((1 << 64) - 1)
            hit |= m
        if hit:
            v[ei][li] = i
    return [v[i >> 6][i & 63] for i in range(w)]


def crafted(rng, w, n, kind):
    if kind == "narrow":  # s_i in [i, i + 3]: many value and index collisions
        return [i + rng.randrange(4) for i in range(w)]
    if kind == "same":
        return [w + 5] * w
    if kind == "chain":  # s_i = i + 1: one chain through every index
        return [i + 1 for i in range(w - 1)] + [w - 1]
    if kind == "small":  # values below 2w
        return [rng.randrange(i, 2 * w) for i in range(w)]
    return [rng.randrange(i, n) for i in range(w)]


@pytest.mark.parametrize("w", [2, 3, 5, 63, 64, 65, 66, 75, 100, 114, 128, 129, 131, 149, 192])
@pytest.mark.parametrize("kind", ["narrow", "same", "chain", "small", "full"])
def test_closed_form_matches_serial_loop(w, kind):
    rng = random.Random(w * 31 + len(kind))
    for trial in range(12):
        s = crafted(rng, w, 57637, kind)
        want = H.remove_duplicates(s)
        assert wave_form(s) == want
        assert closed_form(s) == want
        assert closed_form(s, order_rng=rng) == want
        assert len(set(want)) == w  # the result is a support: distinct positions


def test_fixed_weight_support_uses_the_loop():
    se = H.SeedExpander(bytes(40))
    se2 = H.SeedExpander(bytes(40))
    raw = se2.read(4 * 75)
    r = [int.from_bytes(raw[4 * i:4 * i + 4], "little") for i in range(75)]
    s = [i + ((r[i] * (17669 - i)) >> 32) for i in range(75)]
    assert H.fixed_weight_support(se, 17669, 75) == H.remove_duplicates(s) == closed_form(s) == wave_form(s)
