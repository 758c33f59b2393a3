"""BASELINE.json configs[2] on one GPU: ML-KEM-768, 2^24 handshakes in one batch.

The library runs the batch as 16 chunks of 2^20 against one scratch.  Checks:
* every ss_enc == ss_dec over the whole batch, all 2^24 keys distinct;
* an oracle sample at every chunk boundary (k 2^20 - 1, k 2^20) plus the ends,
  KeyGen included, byte-exact;
* per-record digests SHA3-256(ct || ss) from the GPU equal hashlib's on the sample;
* the per-block shard digests of the one-GPU run equal those of simulated 2-, 4- and
  8-way strong splits, each shard generated from its own first global index (what every
  rank of `bench.py --global-log2-batch 24` does), so the digests do not depend on G.
"""
import hashlib

import numpy as np
import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu

ALG = "ML-KEM-768"
LOG2 = 24
SEED = 0x5EED


def _run_shard(eng, first, count):
    """One rank's work: coins from (seed, global index), KeyGen, Encaps, Decaps, record digests."""
    coins = eng.bench_coins(count, 96, SEED, first)
    kc, ec = coins[:, :64].contiguous(), coins[:, 64:].contiguous()
    del coins
    pk, sk = eng.keypair(coins=kc)
    ct, ss = eng.encaps(pk, coins=ec)
    ss2 = eng.decaps(sk, ct)
    rec = eng.digest_rows(ct, ss)
    torch.cuda.synchronize()
    return kc, ec, pk, sk, ct, ss, ss2, rec


def test_configs2_2p24_one_gpu_and_simulated_splits():
    import oracle as orc
    from qrkem.batch import BatchKEM
    from qrkem.shard import DIGEST_BLOCK, block_digests, combine_digests, strong_shard
    n = 1 << LOG2
    eng = BatchKEM(ALG, device=0)
    kc, ec, pk, sk, ct, ss, ss2, rec = _run_shard(eng, 0, n)
    assert bool((ss == ss2).all())
    assert torch.unique(ss[:, :8].contiguous().view(torch.int64).flatten()).numel() == n
    edges = [k * DIGEST_BLOCK + d for k in range(1, n // DIGEST_BLOCK) for d in (-1, 0)]
    idx = np.unique(np.r_[0:4, edges, n - 4:n])
    ti = torch.from_numpy(idx).cuda()
    kc_h, ec_h, pk_h, sk_h, ct_h, ss_h, rec_h = (t.index_select(0, ti).cpu().numpy()
                                                 for t in (kc, ec, pk, sk, ct, ss, rec))
    opk, osk = orc.batch_keypair(ALG, np.ascontiguousarray(kc_h))
    oct_, oss = orc.batch_encaps(ALG, opk, np.ascontiguousarray(ec_h))
    assert np.array_equal(pk_h, opk) and np.array_equal(sk_h, osk)
    assert np.array_equal(ct_h, oct_) and np.array_equal(ss_h, oss)
    for r, c, s in zip(rec_h, oct_, oss):
        assert r.tobytes() == hashlib.sha3_256(c.tobytes() + s.tobytes()).digest()
    one = block_digests(rec.cpu().numpy(), 0)
    assert len(one) == n // DIGEST_BLOCK
    want = combine_digests(one)
    del kc, ec, pk, sk, ct, ss, ss2, rec
    torch.cuda.empty_cache()
    for world in (2, 4, 8):
        blocks = {}
        for rank in range(world):
            sh = strong_shard(rank, world, n)
            rec = _run_shard(eng, sh.first, sh.count)[-1]  # the other tensors are released here
            blocks.update(block_digests(rec.cpu().numpy(), sh.first))
            del rec
            torch.cuda.empty_cache()
        assert blocks == one, world
        assert combine_digests(blocks) == want


def test_digest_rows_matches_hashlib_on_odd_lengths():
    """The record digest for lengths that are not word multiples (HQC-sized ct, 64-B ss)."""
    from qrkem.batch import BatchKEM
    eng = BatchKEM(ALG, device=0)
    g = torch.Generator().manual_seed(3)
    for la, lb in ((4433, 64), (135, 0), (136, 0), (1088, 32), (1, 7)):
        a = torch.randint(0, 256, (37, la), dtype=torch.uint8, generator=g)
        b = torch.randint(0, 256, (37, lb), dtype=torch.uint8, generator=g) if lb else None
        out = eng.digest_rows(a.cuda(), b.cuda() if b is not None else None).cpu().numpy()
        for i in range(37):
            msg = a[i].numpy().tobytes() + (b[i].numpy().tobytes() if b is not None else b"")
            assert out[i].tobytes() == hashlib.sha3_256(msg).digest(), (la, lb, i)
