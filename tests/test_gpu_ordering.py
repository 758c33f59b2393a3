"""GPU: calls on one context are ordered even when they run on different streams.

A BatchKEM sends device tensors down the stream-ordered device API on the caller's
torch stream and host arrays down the host API on the context's own I/O stream; both
use the context's scratch.  Each call's stream waits for the previous call on the
context (qrk_ctx's last-use event), so a host Encaps issued right after an
asynchronous device KeyGen -- no synchronize in between -- must not overwrite the
KeyGen's scratch.  Both results are checked byte-for-byte against the oracle.
"""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu

ALG = "ML-KEM-768"


def test_device_keypair_then_host_encaps_without_sync():
    """m > mlkem_small_max() (1024): the host Encaps takes the batched path through the packed
    device I/O buffer and the context scratch on the I/O stream (batches up to 1024 run on the
    zero-copy one-launch kernels, which never touch the scratch)."""
    import oracle as orc
    from qrkem.batch import BatchKEM
    n, m = 1 << 16, 2048
    eng = BatchKEM(ALG, device=0)
    coins = orc.bench_coins(n, 64, seed=77)
    host_kc = orc.bench_coins(m, 96, seed=78)
    hpk, _ = orc.batch_keypair(ALG, np.ascontiguousarray(host_kc[:, :64]))
    dcoins = torch.from_numpy(coins).cuda()
    torch.cuda.synchronize()
    pk, sk = eng.keypair(coins=dcoins)                       # async on the torch stream
    ct_h, ss_h = eng.encaps(hpk, coins=np.ascontiguousarray(host_kc[:, 64:]))  # host API, own stream
    torch.cuda.synchronize()
    oct_, oss = orc.batch_encaps(ALG, hpk, np.ascontiguousarray(host_kc[:, 64:]))
    assert np.array_equal(ct_h, oct_) and np.array_equal(ss_h, oss)
    idx = np.unique(np.r_[0:8, 0:n:997, n - 8:n])
    opk, osk = orc.batch_keypair(ALG, np.ascontiguousarray(coins[idx]))
    ti = torch.from_numpy(idx).cuda()
    assert np.array_equal(pk.index_select(0, ti).cpu().numpy(), opk)
    assert np.array_equal(sk.index_select(0, ti).cpu().numpy(), osk)


def test_two_device_streams_on_one_context():
    """KeyGen on a side stream, then Encaps of earlier keys on the default stream."""
    import oracle as orc
    from qrkem.batch import BatchKEM
    n = 1 << 15
    eng = BatchKEM(ALG, device=0)
    c0 = orc.bench_coins(n, 96, seed=5)
    c1 = orc.bench_coins(n, 64, seed=6)
    pk0, _ = eng.keypair(coins=torch.from_numpy(np.ascontiguousarray(c0[:, :64])).cuda())
    ec = torch.from_numpy(np.ascontiguousarray(c0[:, 64:])).cuda()
    d1 = torch.from_numpy(c1).cuda()
    torch.cuda.synchronize()
    side = torch.cuda.Stream()
    with torch.cuda.stream(side):
        pk1, sk1 = eng.keypair(coins=d1)
    ct0, ss0 = eng.encaps(pk0, coins=ec)  # default stream, no wait on `side` by the caller
    torch.cuda.synchronize()
    idx = np.unique(np.r_[0:4, 0:n:1021, n - 4:n])
    ti = torch.from_numpy(idx).cuda()
    opk1, osk1 = orc.batch_keypair(ALG, np.ascontiguousarray(c1[idx]))
    assert np.array_equal(pk1.index_select(0, ti).cpu().numpy(), opk1)
    assert np.array_equal(sk1.index_select(0, ti).cpu().numpy(), osk1)
    opk0, _ = orc.batch_keypair(ALG, np.ascontiguousarray(c0[idx, :64]))
    oct0, oss0 = orc.batch_encaps(ALG, opk0, np.ascontiguousarray(c0[idx, 64:]))
    assert np.array_equal(ct0.index_select(0, ti).cpu().numpy(), oct0)
    assert np.array_equal(ss0.index_select(0, ti).cpu().numpy(), oss0)


def test_device_keypair_then_frodo_host_encaps_without_sync():
    """FrodoKEM has no zero-copy path: even 8 host Encaps run through the context scratch, so
    they must wait for the asynchronous device KeyGen that is still using it."""
    import oracle as orc
    from qrkem.batch import BatchKEM
    fr = "FrodoKEM-640-SHAKE"
    n, m = 1 << 12, 8
    eng = BatchKEM(fr, device=0)
    coins = orc.bench_coins(n, eng.kp_coins, seed=79)
    kc = orc.bench_coins(m, eng.kp_coins, seed=80)
    ec = np.ascontiguousarray(orc.bench_coins(m, eng.enc_coins, seed=81))
    hpk, _ = orc.batch_keypair(fr, np.ascontiguousarray(kc))
    dcoins = torch.from_numpy(coins).cuda()
    torch.cuda.synchronize()
    pk, sk = eng.keypair(coins=dcoins)          # async on the torch stream
    ct_h, ss_h = eng.encaps(hpk, coins=ec)       # host API, own stream, same scratch
    torch.cuda.synchronize()
    oct_, oss = orc.batch_encaps(fr, hpk, ec)
    assert np.array_equal(ct_h, oct_) and np.array_equal(ss_h, oss)
    idx = np.unique(np.r_[0:2, 0:n:1021, n - 2:n])
    opk, osk = orc.batch_keypair(fr, np.ascontiguousarray(coins[idx]))
    ti = torch.from_numpy(idx).cuda()
    assert np.array_equal(pk.index_select(0, ti).cpu().numpy(), opk)
    assert np.array_equal(sk.index_select(0, ti).cpu().numpy(), osk)


def test_host_single_shot_then_device_calls_without_sync():
    """Host-pointer calls run on the context's I/O stream, device-pointer calls on the torch
    stream; each waits for the other through the context's last-use event (abi.cpp LastUse /
    ctx_order).  Single-shot host calls (the pipelined KeyGen uses the context scratch)
    interleaved with device-pointer calls, no synchronize in between, then a host batch large
    enough to regrow the pinned mirror (ctx_quiesce): every output byte-exact vs the oracle."""
    import oracle as orc
    from qrkem.batch import BatchKEM
    n = 1 << 13
    eng = BatchKEM(ALG, device=0)
    for it in range(3):
        kc = np.ascontiguousarray(orc.bench_coins(1, 64, seed=300 + it))
        ec = np.ascontiguousarray(orc.bench_coins(1, 32, seed=310 + it))
        dkc = orc.bench_coins(n, 96, seed=320 + it)
        d_kc = torch.from_numpy(np.ascontiguousarray(dkc[:, :64])).cuda()
        d_ec = torch.from_numpy(np.ascontiguousarray(dkc[:, 64:])).cuda()
        torch.cuda.synchronize()
        hpk, hsk = eng.keypair(coins=kc)            # host, n = 1: I/O stream, context scratch
        pk, sk = eng.keypair(coins=d_kc)            # torch stream, same scratch
        hct, hss = eng.encaps(hpk, coins=ec)        # host single-shot again
        ct_, ss = eng.encaps(pk, coins=d_ec)        # torch stream
        hss2 = eng.decaps(hsk, hct)                 # host single-shot
        ss2 = eng.decaps(sk, ct_)                   # torch stream
        torch.cuda.synchronize()
        opk, osk = orc.batch_keypair(ALG, kc)
        oct_, oss = orc.batch_encaps(ALG, opk, ec)
        assert np.array_equal(hpk, opk) and np.array_equal(hsk, osk)
        assert np.array_equal(hct, oct_) and np.array_equal(hss, oss) and np.array_equal(hss2, oss)
        assert torch.equal(ss, ss2)
        idx = np.unique(np.r_[0:4, 0:n:509, n - 4:n])
        ti = torch.from_numpy(idx).cuda()
        dpk, dsk = orc.batch_keypair(ALG, np.ascontiguousarray(dkc[idx, :64]))
        dct, dss = orc.batch_encaps(ALG, dpk, np.ascontiguousarray(dkc[idx, 64:]))
        assert np.array_equal(sk.index_select(0, ti).cpu().numpy(), dsk)
        assert np.array_equal(ct_.index_select(0, ti).cpu().numpy(), dct)
        assert np.array_equal(ss2.index_select(0, ti).cpu().numpy(), dss)
    # a host batch of 3000 regrows the pinned I/O mirror (waits for the last use first)
    m = 3000
    c3 = orc.bench_coins(m, 96, seed=330)
    pk3, sk3 = eng.keypair(coins=np.ascontiguousarray(c3[:, :64]))
    sel = np.r_[0:3, m - 3:m]
    opk3, osk3 = orc.batch_keypair(ALG, np.ascontiguousarray(c3[sel, :64]))
    assert np.array_equal(pk3[sel], opk3) and np.array_equal(sk3[sel], osk3)


def _residue(ctx):
    import ctypes as ct
    from qrkem._native import LIB
    out = (ct.c_uint64 * 3)()
    assert LIB.qrk_ctx_staging_residue(ctx, out) == 0
    return list(out)


def test_os_coins_staging_wiped():
    """coins=None draws KeyGen seeds / Encaps messages from the OS into pinned host staging and
    uploads them to device staging; both copies are zero when the call returns."""
    from qrkem.batch import BatchKEM
    eng = BatchKEM(ALG, device=0)
    pk, sk = eng.keypair(n=4096)          # batched path, OS coins
    torch.cuda.synchronize()
    h, d, _ = _residue(eng._ctx)
    assert (h, d) == (0, 0)
    ct_, ss = eng.encaps(pk)               # OS Encaps messages
    assert bool((eng.decaps(sk, ct_) == ss).all())
    h, d, _ = _residue(eng._ctx)
    assert (h, d) == (0, 0)


@pytest.mark.parametrize("alg", ["ML-KEM-512", "ML-KEM-768", "ML-KEM-1024"])
def test_mlkem_records_wiped(alg):
    """The batched ML-KEM path leaves no per-handshake key material (r / sigma, m', K', Kbar) in
    scratch once a call has completed (mlkem_cleanse after every chunk, stream-ordered)."""
    import ctypes as ct
    from qrkem._native import LIB
    from qrkem.batch import BatchKEM
    n = 5000  # batched (above the one-launch sizes), ragged
    eng = BatchKEM(alg, device=0)
    fn = LIB.qrk_dbg_mlkem_records_residue
    fn.argtypes = [ct.c_void_p, ct.c_char_p, ct.c_size_t, ct.POINTER(ct.c_uint64)]
    out = ct.c_uint64()

    def residue():
        torch.cuda.synchronize()
        assert fn(eng._ctx, alg.encode(), n, ct.byref(out)) == 0
        return out.value

    pk, sk = eng.keypair(n=n)
    assert residue() == 0
    ct_, ss = eng.encaps(pk)
    assert residue() == 0
    bad = ct_.clone()
    eng.tamper(bad, seed=5, mode=2)  # implicit rejection selects Kbar for half of them
    ss2 = eng.decaps(sk, bad)
    assert residue() == 0
    flip = (bad != ct_).any(dim=1)
    assert bool((ss2[~flip] == ss[~flip]).all()) and not bool((ss2[flip] == ss[flip]).all(dim=1).any())
    eng.close()


def test_cleanse_and_device_restore():
    """qrk_ctx_cleanse zeroes the scratch; a call leaves the caller's current device as it was."""
    from qrkem._native import LIB
    from qrkem.batch import BatchKEM
    eng = BatchKEM(ALG, device=0)
    pk, sk = eng.keypair(n=4096)           # batched: the scratch now holds SampleNTT / PRF output
    ct_, ss = eng.encaps(pk)
    assert bool((eng.decaps(sk, ct_) == ss).all())
    assert _residue(eng._ctx)[2] > 0
    assert LIB.qrk_ctx_cleanse(eng._ctx) == 0
    assert _residue(eng._ctx) == [0, 0, 0]
    assert torch.cuda.current_device() == 0


@pytest.mark.skipif(not torch.cuda.is_available() or torch.cuda.device_count() < 2,
                    reason="needs a second GPU")
def test_context_on_other_device_restores_current():
    """A context on GPU 1 used while GPU 0 is current: every call restores GPU 0 (DeviceGuard)."""
    from qrkem.batch import BatchKEM
    torch.cuda.set_device(0)
    eng = BatchKEM(ALG, device=1)
    pk, sk = eng.keypair(n=64)
    assert torch.cuda.current_device() == 0
    ct_, ss = eng.encaps(pk)
    assert torch.cuda.current_device() == 0
    assert bool((eng.decaps(sk, ct_) == ss).all())
    assert torch.cuda.current_device() == 0


def test_set_chunk_concurrent_with_effective_chunk():
    """qrk_ctx_set_chunk writes the chunk size under the context lock, as qrk_ctx_effective_chunk
    reads it: threads setting two sizes while others read never see any other value."""
    import threading

    from qrkem._native import LIB
    from qrkem.batch import BatchKEM
    eng = BatchKEM(ALG, device=0)
    sizes = (1 << 12, (1 << 20) + 64 * 3)
    seen, stop = set(), threading.Event()

    def setter(k):
        for i in range(4000):
            LIB.qrk_ctx_set_chunk(eng._ctx, sizes[(i + k) & 1])
        stop.set()

    def reader():
        while not stop.is_set():
            seen.add(int(LIB.qrk_ctx_effective_chunk(eng._ctx, ALG.encode())))

    ts = [threading.Thread(target=setter, args=(k,)) for k in range(2)] + [threading.Thread(target=reader) for _ in range(2)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert seen and seen <= set(sizes), seen
