"""HIP ML-KEM parity vs the oracle, through the C ABI (libqrkem.so).

Bar: byte-exact pk / sk / ct / ss for every index (integer work).
Sizes are ragged on purpose (not multiples of the 16-handshake workgroup or
the 64-instance scratch tile).
"""
import hashlib

import numpy as np
import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu

ALGS = ["ML-KEM-512", "ML-KEM-768", "ML-KEM-1024"]


@pytest.fixture(scope="module")
def engines():
    from qrkem.batch import BatchKEM
    return {a: BatchKEM(a, device=0) for a in ALGS}


def _dev(a):
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


def _host(t):
    torch.cuda.synchronize()
    return t.cpu().numpy()


@pytest.mark.parametrize("alg", ALGS)
@pytest.mark.parametrize("n", [1, 2, 16, 17, 255, 256, 257, 301, 1024, 1025])
def test_roundtrip_matches_oracle(engines, alg, n):
    """n <= 1024 runs the one-launch small-batch kernels (KeyGen: one workgroup per item for
    n <= 16, k_keygen_multi, then one per handshake), n > 1024 the batched schedule; both
    byte-exact vs the oracle, including the boundaries."""
    import oracle as orc
    eng = engines[alg]
    coins = orc.bench_coins(n, 96, seed=1234 + n)
    kc, ec = np.ascontiguousarray(coins[:, :64]), np.ascontiguousarray(coins[:, 64:])
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
def test_tampered_implicit_rejection(engines, alg):
    import oracle as orc
    eng = engines[alg]
    n = 130
    coins = orc.bench_coins(n, 96, seed=99)
    kc, ec = np.ascontiguousarray(coins[:, :64]), np.ascontiguousarray(coins[:, 64:])
    opk, osk = orc.batch_keypair(alg, kc)
    oct_, oss = orc.batch_encaps(alg, opk, ec)
    bad = oct_.copy()
    rng = np.random.default_rng(7)
    flip = rng.random(n) < 0.5
    for i in np.nonzero(flip)[0]:
        bit = int(rng.integers(0, 8 * bad.shape[1]))
        bad[i, bit // 8] ^= 1 << (bit % 8)
    ss = _host(eng.decaps(_dev(osk), _dev(bad)))
    want = orc.batch_decaps(alg, osk, bad)
    assert np.array_equal(ss, want)
    assert np.array_equal(ss[~flip], oss[~flip])
    assert not np.any(np.all(ss[flip] == oss[flip], axis=1))


@pytest.mark.parametrize("alg", ALGS)
@pytest.mark.parametrize("n", [(1 << 15) - 5, (1 << 15) + 1])
def test_pair_front_boundary(engines, alg, n):
    """Chunks of at most 2^15 handshakes run two sponge fronts, Encaps' H(ek) + G and Decaps'
    G(m' || h), on lane pairs (csrc/keccak_pair.cuh; J(z || c) stays one lane per handshake), larger
    chunks one lane per handshake: both sides of the
    boundary byte-exact vs the oracle on a sample of indices (both ends included), Decaps with a
    quarter of the ciphertexts tampered."""
    import oracle as orc
    eng = engines[alg]
    coins = orc.bench_coins(n, 96, seed=4242 + n)
    kc, ec = np.ascontiguousarray(coins[:, :64]), np.ascontiguousarray(coins[:, 64:])
    pk, sk = eng.keypair(coins=_dev(kc))
    ct, ss = eng.encaps(pk, coins=_dev(ec))
    bad = _host(ct).copy()
    flip = (np.arange(n) % 4) == 1
    bad[flip, 7] ^= 0x20
    ss2 = _host(eng.decaps(sk, _dev(bad)))
    pk, sk, ct, ss = map(_host, (pk, sk, ct, ss))
    idx = np.unique(np.concatenate([np.arange(8), n - 1 - np.arange(8), np.linspace(0, n - 1, 200).astype(int)]))
    opk, osk = orc.batch_keypair(alg, np.ascontiguousarray(kc[idx]))
    assert np.array_equal(pk[idx], opk) and np.array_equal(sk[idx], osk)
    oct_, oss = orc.batch_encaps(alg, opk, np.ascontiguousarray(ec[idx]))
    assert np.array_equal(ct[idx], oct_) and np.array_equal(ss[idx], oss)
    assert np.array_equal(ss2[idx], orc.batch_decaps(alg, osk, np.ascontiguousarray(bad[idx])))
    assert np.array_equal(ss2[~flip], ss[~flip])


@pytest.mark.parametrize("alg", ALGS)
@pytest.mark.parametrize("n", [5, 16, 17])
def test_host_pointer_api(engines, alg, n):
    """Host-array calls: n <= 16 KeyGens run the pipelined kernel (k_keygen_pipe, its error word
    checked), n = 17 the one-workgroup-per-handshake kernel; Encaps / Decaps the one-launch kernels."""
    import oracle as orc
    eng = engines[alg]
    coins = orc.bench_coins(n, 96, seed=5 + n)
    kc, ec = np.ascontiguousarray(coins[:, :64]), np.ascontiguousarray(coins[:, 64:])
    pk, sk = eng.keypair(coins=kc)
    ct, ss, st = eng.encaps(pk, coins=ec, return_status=True)
    assert np.all(st == 0)
    opk, osk = orc.batch_keypair(alg, kc)
    oct_, oss = orc.batch_encaps(alg, opk, ec)
    assert np.array_equal(pk, opk) and np.array_equal(sk, osk)
    assert np.array_equal(ct, oct_) and np.array_equal(ss, oss)
    assert np.array_equal(eng.decaps(sk, ct), oss)


def test_modulus_check_status(engines):
    import oracle as orc
    alg = "ML-KEM-768"
    eng = engines[alg]
    coins = orc.bench_coins(4, 96, seed=11)
    opk, _ = orc.batch_keypair(alg, np.ascontiguousarray(coins[:, :64]))
    pk = opk.copy()
    pk[1, 0] = 0xFF
    pk[1, 1] |= 0x0F  # first coefficient = 4095 >= q
    _, _, st = eng.encaps(_dev(pk), coins=_dev(np.ascontiguousarray(coins[:, 64:])), return_status=True)
    st = _host(st)
    assert list(st) == [0, -1, 0, 0]


def test_single_shot_oqs_api():
    import oracle as orc
    from qrkem import oqs
    alg = "ML-KEM-768"
    kc = bytes(range(64))
    ec = bytes(range(100, 132))
    k = oqs.KeyEncapsulation(alg)
    pk = k.generate_keypair_derand(kc)
    sk = k.export_secret_key()
    opk, osk = orc.keypair(alg, kc)
    assert pk == opk and sk == osk
    c, ss = oqs.KeyEncapsulation(alg).encap_secret_derand(pk, ec)
    oc, oss = orc.encaps(alg, pk, ec)
    assert c == oc and ss == oss
    assert oqs.KeyEncapsulation(alg, sk).decap_secret(c) == oss
    # random (OS CSPRNG) path round-trips
    pk2 = k.generate_keypair()
    c2, s2 = oqs.KeyEncapsulation(alg).encap_secret(pk2)
    assert oqs.KeyEncapsulation(alg, k.export_secret_key()).decap_secret(c2) == s2


@pytest.mark.parametrize("alg", ALGS)
def test_single_shot_paths_all_params(alg):
    """The n = 1 one-launch kernels through the OQS API (zero-copy pinned I/O, completion flag):
    byte-exact KeyGen / Encaps / Decaps, implicit rejection of a tampered ciphertext (ss = J(z || c)
    from the oracle), and the FIPS 203 modulus check raising RuntimeError, repeated so the flag
    tickets and the reused pinned mirror are exercised."""
    import oracle as orc
    from qrkem import oqs
    rng = np.random.default_rng(sum(map(ord, alg)))
    for it in range(4):
        kc = rng.integers(0, 256, 64, dtype=np.uint8).tobytes()
        ec = rng.integers(0, 256, 32, dtype=np.uint8).tobytes()
        k = oqs.KeyEncapsulation(alg)
        pk = k.generate_keypair_derand(kc)
        sk = k.export_secret_key()
        opk, osk = orc.keypair(alg, kc)
        assert pk == opk and sk == osk
        c, ss = oqs.KeyEncapsulation(alg).encap_secret_derand(pk, ec)
        oc, oss = orc.encaps(alg, pk, ec)
        assert c == oc and ss == oss
        assert oqs.KeyEncapsulation(alg, sk).decap_secret(c) == oss
        bad = bytearray(c)
        bad[(17 * it) % len(bad)] ^= 1 << it
        want = orc.batch_decaps(alg, np.frombuffer(sk, np.uint8).reshape(1, -1),
                                np.frombuffer(bytes(bad), np.uint8).reshape(1, -1))[0].tobytes()
        got = oqs.KeyEncapsulation(alg, sk).decap_secret(bytes(bad))
        assert got == want and got != oss
    badpk = bytearray(pk)
    badpk[0] = 0xFF
    badpk[1] |= 0x0F  # first coefficient 4095 >= q
    with pytest.raises(RuntimeError):
        oqs.KeyEncapsulation(alg).encap_secret(bytes(badpk))


def test_bench_coins_device_matches_oracle(engines):
    import oracle as orc
    eng = engines["ML-KEM-768"]
    got = _host(eng.bench_coins(1000, 96, seed=0x5EED, first=12345))
    assert np.array_equal(got, orc.bench_coins(1000, 96, 0x5EED, 12345))


def test_tamper_kernel_matches_definition(engines):
    eng = engines["ML-KEM-768"]
    n, L = 200, 1088
    base = np.zeros((n, L), np.uint8)
    t = _dev(base)
    eng.tamper(t, seed=77, mode=2)
    got = _host(t)
    for i in range(n):
        h = int.from_bytes(hashlib.shake_256(b"qrk-tamper" + (77).to_bytes(8, "little")
                                             + i.to_bytes(8, "little")).digest(8), "little")
        want = np.zeros(L, np.uint8)
        if h & 1:
            bit = (h >> 1) % (8 * L)
            want[bit // 8] = 1 << (bit % 8)
        assert np.array_equal(got[i], want), i


@pytest.mark.parametrize("alg", ALGS)
def test_kat_drbg_records_match_golden(engines, golden_dir, alg):
    """BASELINE.json configs[0] on the GPU: every NIST-KAT-DRBG record (1024 for
    ML-KEM-768) byte-exact against the golden digests of the Python restatement."""
    import json
    import oracle as orc
    g = json.loads((golden_dir / "kat_mlkem.json").read_text())[alg]
    n = g["count"]
    _, kc, ec = orc.kat_coins(n, 64, 32)
    eng = engines[alg]
    pk, sk = eng.keypair(coins=_dev(kc))
    ct, ss = eng.encaps(pk, coins=_dev(ec))
    ss2 = eng.decaps(sk, ct)
    pk, sk, ct, ss, ss2 = map(_host, (pk, sk, ct, ss, ss2))
    assert np.array_equal(ss, ss2)
    for name, arr in (("pk", pk), ("sk", sk), ("ct", ct), ("ss", ss)):
        assert hashlib.sha256(arr.tobytes()).hexdigest() == g["digests"][name], name


def test_large_batch_roundtrip_and_sample(engines):
    """2^16 handshakes (several chunks with a small chunk size): every ss_enc == ss_dec,
    a stride sample byte-exact vs the oracle."""
    import oracle as orc
    from qrkem.batch import BatchKEM
    alg, n = "ML-KEM-768", 1 << 16
    eng = BatchKEM(alg, device=0, chunk=10000)
    coins = eng.bench_coins(n, 96, seed=42)
    kc, ec = coins[:, :64].contiguous(), coins[:, 64:].contiguous()
    pk, sk = eng.keypair(coins=kc)
    ct, ss = eng.encaps(pk, coins=ec)
    ss2 = eng.decaps(sk, ct)
    torch.cuda.synchronize()
    assert bool((ss == ss2).all())
    idx = np.r_[0:64, 9999:10003, 4096:n:4096, n - 5:n]
    pk_h, sk_h, ct_h, ss_h = (t.cpu().numpy()[idx] for t in (pk, sk, ct, ss))
    kc_h, ec_h = kc.cpu().numpy()[idx], ec.cpu().numpy()[idx]
    opk, osk = orc.batch_keypair(alg, np.ascontiguousarray(kc_h))
    oct_, oss = orc.batch_encaps(alg, opk, np.ascontiguousarray(ec_h))
    assert np.array_equal(pk_h, opk) and np.array_equal(sk_h, osk)
    assert np.array_equal(ct_h, oct_) and np.array_equal(ss_h, oss)


@pytest.mark.parametrize("alg", ALGS)
def test_kat_records_through_single_shot_wrapper(golden_dir, alg):
    """BASELINE.json configs[0] as the reference runs it: one KEM object and one call per
    handshake through the oqs-compatible wrapper (qrkem.oqs, the drop-in for vendor/oqs.py),
    every NIST-KAT-DRBG record (1024 for ML-KEM-768), digests equal to the golden ones; KeyGen
    runs the pipelined single-shot kernel (k_keygen_pipe), Encaps / Decaps the one-launch kernels."""
    import json
    import oracle as orc
    from qrkem import oqs
    g = json.loads((golden_dir / "kat_mlkem.json").read_text())[alg]
    n = g["count"]
    _, kc, ec = orc.kat_coins(n, 64, 32)
    h = {k: hashlib.sha256() for k in ("pk", "sk", "ct", "ss")}
    for i in range(n):
        kem = oqs.KeyEncapsulation(alg)
        pk = kem.generate_keypair_derand(kc[i].tobytes())
        sk = kem.export_secret_key()
        c, ss = oqs.KeyEncapsulation(alg).encap_secret_derand(pk, ec[i].tobytes())
        assert oqs.KeyEncapsulation(alg, sk).decap_secret(c) == ss
        for k, v in (("pk", pk), ("sk", sk), ("ct", c), ("ss", ss)):
            h[k].update(v)
    for k in h:
        assert h[k].hexdigest() == g["digests"][k], k


def _sample_ntt_needs_4th_block(rho: bytes, i: int, j: int) -> bool:
    """FIPS 203 Alg. 7 acceptance count over the first 3 SHAKE128 blocks (504 bytes)."""
    b = hashlib.shake_128(rho + bytes([j, i])).digest(504)
    cnt = 0
    for t in range(0, 504, 3):
        d1 = b[t] | ((b[t + 1] & 0x0F) << 8)
        d2 = (b[t + 1] >> 4) | (b[t + 2] << 4)
        cnt += (d1 < 3329) + (d2 < 3329)
    return cnt < 256


@pytest.mark.parametrize("alg,k,n", [("ML-KEM-768", 3, 1100), ("ML-KEM-512", 2, 1100),
                                     # half a chunk: >= 2^19 entries on one fix-up list
                                     ("ML-KEM-768", 3, (1 << 19) + 3)])
def test_sample_ntt_fixup_resume_and_overflow(engines, alg, k, n):
    """Every pk of a batch carries a rho whose matrix has entries that need a 4th SHAKE128 block,
    so every handshake has entries on the SampleNTT fix-up list (far more than the ~0.7 % of random
    keys).  Encaps is byte-exact vs the oracle for every index (a stride sample of the full chunk)."""
    import oracle as orc
    rng = np.random.default_rng(77 + k)
    for _ in range(4000):
        rho = bytes(rng.integers(0, 256, 32, dtype=np.uint8))
        bad = sum(_sample_ntt_needs_4th_block(rho, i, j) for i in range(k) for j in range(k))
        if bad >= 1:
            break
    else:
        pytest.fail("no rho with a 4-block SampleNTT entry found")
    # n > 1024: the batched schedule (k_xof + k_xof_fix)
    coins = orc.bench_coins(n, 96, seed=4242)
    kc, ec = np.ascontiguousarray(coins[:, :64]), np.ascontiguousarray(coins[:, 64:])
    opk, _ = orc.batch_keypair(alg, kc[:1])
    pk = np.repeat(opk, n, axis=0)
    pk[:, -32:] = np.frombuffer(rho, dtype=np.uint8)
    eng = engines[alg]
    ct, ss = eng.encaps(_dev(pk), coins=_dev(ec))
    idx = np.arange(n) if n <= 4096 else np.unique(np.r_[np.arange(0, n, 257), n - 1])
    oct_, oss = orc.batch_encaps(alg, pk[idx], np.ascontiguousarray(ec[idx]), 8)
    assert np.array_equal(_host(ct)[idx], oct_)
    assert np.array_equal(_host(ss)[idx], oss)


@pytest.mark.parametrize("alg,k", [("ML-KEM-512", 2), ("ML-KEM-768", 3), ("ML-KEM-1024", 4)])
def test_fixup_counters_across_calls(alg, k):
    """Chunks of at most 2^15 read rho from the keys and count SampleNTT fix-ups into one of the
    context's two counters, each call zeroing the other for the next (no k_rho_copy launch).  A run of
    Encaps / Decaps calls whose every pk needs fix-ups -- direct-path chunks back to back, a call split
    into several direct chunks, and copy-path chunks (> 2^15) in between -- stays byte-exact vs the
    oracle on every call (Decaps with dk's copy of rho replaced too)."""
    import oracle as orc
    from qrkem.batch import BatchKEM
    rng = np.random.default_rng(91 + k)
    for _ in range(4000):
        rho = bytes(rng.integers(0, 256, 32, dtype=np.uint8))
        if sum(_sample_ntt_needs_4th_block(rho, i, j) for i in range(k) for j in range(k)) >= 1:
            break
    else:
        pytest.fail("no rho with a 4-block SampleNTT entry found")
    kc0 = np.ascontiguousarray(orc.bench_coins(1, 64, seed=91))
    opk, osk = orc.batch_keypair(alg, kc0)
    opk[:, -32:] = np.frombuffer(rho, dtype=np.uint8)
    osk[:, 768 * k:768 * k + 32] = np.frombuffer(rho, dtype=np.uint8)  # dk's copy of ek's rho (H(ek) stale)
    big = BatchKEM(alg, device=0)
    small = BatchKEM(alg, device=0, chunk=2048)  # a 5000-handshake call = three direct-path chunks
    for step, (eng, n) in enumerate([(big, 1100), (big, 3000), (small, 5000), (big, (1 << 15) + 64), (big, 1500),
                                     (small, 5000), (big, 2000)]):
        coins = orc.bench_coins(n, 32, seed=300 + step)
        pk = np.repeat(opk, n, axis=0)
        sk = np.repeat(osk, n, axis=0)
        ct, ss = eng.encaps(_dev(pk), coins=_dev(coins))
        ss2 = _host(eng.decaps(_dev(sk), ct))
        ct, ss = _host(ct), _host(ss)
        idx = np.unique(np.r_[np.arange(4), np.linspace(0, n - 1, 120).astype(int), n - 1])
        oct_, oss = orc.batch_encaps(alg, pk[idx], np.ascontiguousarray(coins[idx]))
        assert np.array_equal(ct[idx], oct_), (step, n)
        assert np.array_equal(ss[idx], oss), (step, n)
        # Decaps re-encrypts under the same fix-up-heavy rho (its implicit-rejection outcome as the oracle's)
        assert np.array_equal(ss2[idx], orc.batch_decaps(alg, sk[idx], np.ascontiguousarray(ct[idx]))), (step, n)


# (alg, workgroup role): roles < 2K are PRF items (NTT(s_j) operands, NTT(e_i)), roles 2K .. 3K - 2 the
# t_hat rows 1 .. K - 1, whose late t_hat flag the collector would otherwise take from the stale word
@pytest.mark.parametrize("alg,item", [("ML-KEM-512", 0), ("ML-KEM-512", 4), ("ML-KEM-768", 0), ("ML-KEM-768", 5),
                                      ("ML-KEM-768", 7), ("ML-KEM-1024", 7), ("ML-KEM-1024", 10)])
def test_keygen_pipe_forced_timeout(engines, alg, item):
    """The pipelined single-shot KeyGen (k_keygen_pipe, host-pointer calls of n <= 16) under a lost
    hand-off: the workgroup of role `item` (a PRF item or a t_hat row) publishes its payload and flags
    150 ms late, past every consumer's and the collector's 50 ms bounded wait (debug knob
    qrk_dbg_kg_late).  The call must fail (OQS_ERROR -> RuntimeError, as vendor/oqs.py:323-326 raises
    for the reference), never return keys; the straggler's flags, set after the collector's reset,
    must not poison the next call, which is byte-exact vs the oracle (single-shot and a 3-handshake
    host batch), and the context's flag words are all zero again after the failed call (a build
    without the host's re-zeroing leaves the straggler's flags set, profiles/r6/single_shot/)."""
    import ctypes as ct
    import oracle as orc
    from qrkem import oqs
    from qrkem._native import LIB, last_error
    dbg = LIB.qrk_dbg_kg_late
    dbg.argtypes, dbg.restype = [ct.c_int], ct.c_int
    rng = np.random.default_rng(item + 31 * len(alg))
    kc, kc_lost = (rng.integers(0, 256, 64, dtype=np.uint8).tobytes() for _ in range(2))
    kcb, kcb_lost = (rng.integers(0, 256, (3, 64), dtype=np.uint8) for _ in range(2))
    eng = engines[alg]
    # the failing calls use other coins than the recovery calls, so a stale flag that let the next
    # call read the straggler's payload would show up as wrong keys
    try:
        dbg(item)
        with pytest.raises(RuntimeError):
            oqs.KeyEncapsulation(alg).generate_keypair_derand(kc_lost)
        with pytest.raises(RuntimeError):
            eng.keypair(coins=kcb_lost)
        assert "hand-off timeout" in last_error()
        # the straggler set its flags after the collector's reset; the failed call re-zeroed them
        res = LIB.qrk_dbg_kg_flags_residue
        res.argtypes, res.restype = [ct.c_void_p, ct.POINTER(ct.c_uint64)], ct.c_int
        cnt = ct.c_uint64(1)
        assert res(eng._ctx, ct.byref(cnt)) == 0 and cnt.value == 0
    finally:
        dbg(-1)
    opk, osk = orc.keypair(alg, kc)
    for _ in range(2):
        k = oqs.KeyEncapsulation(alg)
        assert k.generate_keypair_derand(kc) == opk and k.export_secret_key() == osk
        pk, sk = eng.keypair(coins=kcb)
        bpk, bsk = orc.batch_keypair(alg, kcb)
        assert np.array_equal(pk, bpk) and np.array_equal(sk, bsk)


@pytest.mark.parametrize("op", ["encaps", "decaps"])
def test_fixup_counters_rezeroed_after_failed_chunk(op):
    """the two alternating SampleNTT fix-up counters of chunks <= 2^15 stay exact when a
    chunk fails after the parity flip (debug hook qrk_dbg_fail_after_flip: the chunk returns an
    error before its first launch, so its main pass never zeroes the word the next call counts
    into).  The failed call raises; the next call counts exactly n x (its pk's fix-up entries) --
    read back with qrk_dbg_fixc_words -- and is byte-exact vs the oracle.  Without the re-zero the
    word would carry the previous call's count as well."""
    import ctypes as ct
    import oracle as orc
    from qrkem._native import LIB
    from qrkem.batch import BatchKEM
    alg, k = "ML-KEM-768", 3
    rng = np.random.default_rng(1234)
    for _ in range(4000):
        rho = bytes(rng.integers(0, 256, 32, dtype=np.uint8))
        bad = sum(_sample_ntt_needs_4th_block(rho, i, j) for i in range(k) for j in range(k))
        if bad >= 1:
            break
    else:
        pytest.fail("no rho with a 4-block SampleNTT entry found")
    kc0 = np.ascontiguousarray(orc.bench_coins(1, 64, seed=1234))
    opk, osk = orc.batch_keypair(alg, kc0)
    opk[:, -32:] = np.frombuffer(rho, dtype=np.uint8)
    osk[:, 768 * k:768 * k + 32] = np.frombuffer(rho, dtype=np.uint8)
    fail = LIB.qrk_dbg_fail_after_flip
    fail.argtypes, fail.restype = [ct.c_int], ct.c_int
    words = LIB.qrk_dbg_fixc_words
    words.argtypes, words.restype = [ct.c_void_p, ct.POINTER(ct.c_uint32), ct.POINTER(ct.c_int)], ct.c_int
    eng = BatchKEM(alg, device=0)

    def run(n, seed):
        coins = orc.bench_coins(n, 32, seed=seed)
        pk, sk = np.repeat(opk, n, axis=0), np.repeat(osk, n, axis=0)
        if op == "encaps":
            ct_, ss = eng.encaps(_dev(pk), coins=_dev(coins))
            return pk, sk, coins, _host(ct_), _host(ss)
        oct_, _ = orc.batch_encaps(alg, pk, coins)
        return pk, sk, coins, oct_, _host(eng.decaps(_dev(sk), _dev(oct_)))

    run(1100, 1)  # counts 1100 * bad into one word
    try:
        fail(1)
        with pytest.raises(RuntimeError):
            run(1200, 2)
    finally:
        fail(0)
    n = 1300
    pk, sk, coins, ct_, ss = run(n, 3)
    w = (ct.c_uint32 * 2)()
    par = ct.c_int()
    assert words(eng._ctx, w, ct.byref(par)) == 0
    assert sorted([w[0], w[1]]) == [0, n * bad], (w[0], w[1], bad)
    idx = np.unique(np.r_[np.arange(4), np.linspace(0, n - 1, 60).astype(int)])
    if op == "encaps":
        oct_, oss = orc.batch_encaps(alg, pk[idx], np.ascontiguousarray(coins[idx]))
        assert np.array_equal(ct_[idx], oct_) and np.array_equal(ss[idx], oss)
    else:
        assert np.array_equal(ss[idx], orc.batch_decaps(alg, sk[idx], np.ascontiguousarray(ct_[idx])))
    eng.close()
