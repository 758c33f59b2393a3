"""The auto schedule (independent kernels of one operation in multi-role launches, every kernel
on the caller's stream) against the serial schedule (one kernel per launch) and the C oracle,
and the asynchrony of the device-pointer API.

Round 3's side-stream schedule produced wrong ciphertexts in every row when KeyGen and Encaps
ran back to back on one context as the first GPU process of a box (DESIGN.md section 1,
"Ordering"); the library now has no side streams at all, and these tests pin both properties the
redesign is for: byte-exact outputs under back-to-back calls with the sampled matrix poisoned
(QRK_DEBUG_POISON, set for the whole GPU suite in conftest.py) and a device call that returns to
the host before its kernels finish.  n = 300000 is a ragged batch (not a multiple of 256); every
stage is compared on its own, so a failure names the stage and counts its mismatching rows.
"""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu

N = 300000
PARTS = 8  # report mismatching rows per eighth of the batch (and check the oracle at its boundaries)


def _boundary_idx(n, parts=PARTS):
    """the ends of the batch and of each eighth (workgroup and tile boundaries among them)"""
    cq = ((n + 63) // 64 * 64) // parts
    idx = [0, 1, 63, 64, 255, 256, n - 1]
    for q in range(1, parts):
        idx += [q * cq - 2, q * cq - 1, q * cq, q * cq + 1]
    return np.unique(np.array([i for i in idx if 0 <= i < n]))


def _rows_per_part(a, b, n=N, parts=PARTS):
    bad = torch.nonzero((a != b).any(dim=1)).flatten().cpu()
    cq = ((n + 63) // 64 * 64) // parts
    return [int(((bad >= q * cq) & (bad < (q + 1) * cq)).sum()) for q in range(parts)], bad[:8].tolist()


@pytest.mark.parametrize("alg,n", [("ML-KEM-768", N), ("ML-KEM-1024", N),
                                   # a ragged batch of more than 2^19 handshakes in one chunk
                                   ("ML-KEM-768", (1 << 19) + 4097)])
def test_back_to_back_auto_vs_serial(alg, n):
    """KeyGen -> Encaps -> tamper -> Decaps on one context with no host synchronisation in
    between, then the same on the serial schedule."""
    from qrkem.batch import BatchKEM
    eng = BatchKEM(alg, device=0)  # default schedule: multi-role launches
    coins = eng.bench_coins(n, 96, seed=400 + len(alg))
    kc, ec = coins[:, :64].contiguous(), coins[:, 64:].contiguous()
    pk, sk = eng.keypair(coins=kc)
    ct, ss = eng.encaps(pk, coins=ec)
    bad = ct.clone()
    eng.tamper(bad, seed=78, mode=2)
    ss2 = eng.decaps(sk, bad)
    torch.cuda.synchronize()
    ser = BatchKEM(alg, device=0)
    ser.set_streams(1)
    pk_s, sk_s = ser.keypair(coins=kc)
    ct_s, ss_s = ser.encaps(pk_s, coins=ec)
    ss2_s = ser.decaps(sk_s, bad)
    torch.cuda.synchronize()
    stages = {k: _rows_per_part(a, b, n) for k, a, b in (("pk", pk, pk_s), ("sk", sk, sk_s), ("ct", ct, ct_s),
                                                          ("ss", ss, ss_s), ("ss2", ss2, ss2_s))}
    assert all(sum(v[0]) == 0 for v in stages.values()), stages
    del pk, sk, ct, ss, bad, ss2, pk_s, sk_s, ct_s, ss_s, ss2_s, coins, kc, ec
    eng.close()
    ser.close()
    torch.cuda.empty_cache()


@pytest.mark.parametrize("alg", ["ML-KEM-768", "ML-KEM-1024"])
def test_auto_schedule_equals_serial_and_oracle(alg):
    import oracle as orc
    from qrkem.batch import BatchKEM
    eng = BatchKEM(alg, device=0)
    eng.set_streams(0)  # multi-role launches
    ser = BatchKEM(alg, device=0)
    ser.set_streams(1)  # serial schedule: one kernel per launch
    coins = eng.bench_coins(N, 96, seed=300 + len(alg))
    kc, ec = coins[:, :64].contiguous(), coins[:, 64:].contiguous()

    pk, sk = eng.keypair(coins=kc)
    pk_s, sk_s = ser.keypair(coins=kc)
    torch.cuda.synchronize()
    assert torch.equal(pk, pk_s), ("keypair pk", _rows_per_part(pk, pk_s))
    assert torch.equal(sk, sk_s), ("keypair sk", _rows_per_part(sk, sk_s))

    ct, ss = eng.encaps(pk, coins=ec)
    ct_s, ss_s = ser.encaps(pk, coins=ec)
    torch.cuda.synchronize()
    assert torch.equal(ct, ct_s), ("encaps ct", _rows_per_part(ct, ct_s))
    assert torch.equal(ss, ss_s), ("encaps ss", _rows_per_part(ss, ss_s))

    bad = ct.clone()
    eng.tamper(bad, seed=77, mode=2)
    flip = (bad != ct).any(dim=1)
    ss2 = eng.decaps(sk, bad)
    ss2_s = ser.decaps(sk, bad)
    torch.cuda.synchronize()
    assert torch.equal(ss2_s[~flip], ss[~flip]), "serial decaps of untampered rows"
    assert torch.equal(ss2, ss2_s), ("decaps ss", _rows_per_part(ss2, ss2_s))
    assert not bool((ss2[flip] == ss[flip]).all(dim=1).any())

    idx = _boundary_idx(N)
    ti = torch.from_numpy(idx).cuda()
    kc_h, ec_h, ct_h, ss_h, bad_h, ss2_h = (t.index_select(0, ti).cpu().numpy()
                                            for t in (kc, ec, ct, ss, bad, ss2))
    opk, osk = orc.batch_keypair(alg, np.ascontiguousarray(kc_h))
    oct_, oss = orc.batch_encaps(alg, opk, np.ascontiguousarray(ec_h))
    assert np.array_equal(ct_h, oct_) and np.array_equal(ss_h, oss)
    assert np.array_equal(ss2_h, orc.batch_decaps(alg, osk, np.ascontiguousarray(bad_h)))
    del pk, sk, ct, ss, bad, ss2, pk_s, sk_s, ct_s, ss_s, ss2_s, coins, kc, ec
    eng.close()
    ser.close()
    torch.cuda.empty_cache()


def test_device_encaps_returns_before_its_kernels_finish():
    """A 2^20-handshake ML-KEM-768 Encaps on device tensors with device coins is stream-ordered
    and asynchronous (include/qrkem.h): the call returns while its kernels are still running (the
    stream reports busy right after the call, and the call takes a small fraction of the time to
    completion), and its outputs equal a synchronous run's."""
    import time
    from qrkem.batch import BatchKEM
    n = 1 << 20
    eng = BatchKEM("ML-KEM-768", device=0)
    coins = eng.bench_coins(n, 96, seed=4242)
    kc, ec = coins[:, :64].contiguous(), coins[:, 64:].contiguous()
    pk, _ = eng.keypair(coins=kc)
    ct0, ss0 = eng.encaps(pk, coins=ec)  # grows the scratch (host-synchronous allocation)
    torch.cuda.synchronize()
    warm = (torch.empty_like(ct0), torch.empty_like(ss0))  # caching-allocator blocks for the outputs
    del warm
    torch.cuda.synchronize()
    stream = torch.cuda.current_stream()
    t0 = time.perf_counter()
    ct, ss = eng.encaps(pk, coins=ec)
    t1 = time.perf_counter()
    busy = not stream.query()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    assert busy, "the stream was idle when encaps returned: the call waited for its kernels"
    assert (t1 - t0) < 0.5 * (t2 - t0), (t1 - t0, t2 - t0)
    assert torch.equal(ct, ct0) and torch.equal(ss, ss0)
    # scratch of a 2^20 ML-KEM-768 chunk: the batched layout (~5.0 KB per handshake: the 12-bit
    # sampled matrix, PRF words, per-handshake records, fix-up list), not 16 KiB per handshake for
    # the multi-workgroup KeyGen's slots, of which only QRK_KG_MULTI_MAX are used
    assert 4800 * n <= eng.scratch_bytes <= 5200 * n, eng.scratch_bytes
    del pk, ct0, ss0, ct, ss, coins, kc, ec
    eng.close()
    torch.cuda.empty_cache()
