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
    import oracle as orc
    from qrkem.batch import BatchKEM
    n, m = 1 << 16, 300
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


def test_cleanse_and_device_restore():
    """qrk_ctx_cleanse zeroes the scratch; a call leaves the caller's current device as it was."""
    from qrkem._native import LIB
    from qrkem.batch import BatchKEM
    eng = BatchKEM(ALG, device=0)
    pk, sk = eng.keypair(n=128)
    ct_, ss = eng.encaps(pk)
    assert bool((eng.decaps(sk, ct_) == ss).all())
    assert LIB.qrk_ctx_cleanse(eng._ctx) == 0
    assert torch.cuda.current_device() == 0
