"""CPU, world size 2 (gloo): the multi-GPU path's sharding and end-of-run
reduction, exercised with real processes.  Each rank derives its shard's coins
from (seed, global index) and runs the oracle KEM on them (standing in for its
GPU); the test checks that the shards tile the batch, that per-shard bytes do
not depend on the rank count, and that counters / elapsed reduce correctly.
"""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

ALG = "ML-KEM-768"
PER_RANK = 24
SEED = 0x5EED


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, outdir):
    import sys
    from pathlib import Path
    root = Path(__file__).resolve().parents[1]
    sys.path[:0] = [str(root / "quantum-resistant-p2p_amd"), str(root / "oracle")]
    import torch.distributed as dist
    import oracle as orc
    from qrkem.shard import reduce_run, weak_shard
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    sh = weak_shard(rank, world, PER_RANK)
    coins = orc.bench_coins(sh.count, 96, SEED, sh.first)
    pk, sk = orc.batch_keypair(ALG, np.ascontiguousarray(coins[:, :64]), 1)
    ct, ss = orc.batch_encaps(ALG, pk, np.ascontiguousarray(coins[:, 64:]), 1)
    ss2 = orc.batch_decaps(ALG, sk, ct, 1)
    mism = int((ss != ss2).any(axis=1).sum())
    elapsed, (done, bad) = reduce_run(0.5 + rank, [sh.count, mism])
    np.save(os.path.join(outdir, f"ss_{rank}.npy"), ss)
    with open(os.path.join(outdir, f"red_{rank}.txt"), "w") as f:
        f.write(f"{elapsed} {done} {bad} {sh.first}\n")
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_sharding_and_reduce(tmp_path):
    import oracle as orc
    world = 2
    mp.start_processes(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True,
                       start_method="spawn")
    reds = [open(tmp_path / f"red_{r}.txt").read().split() for r in range(world)]
    for r, (elapsed, done, bad, first) in enumerate(reds):
        assert float(elapsed) == 0.5 + (world - 1)  # max over ranks
        assert int(done) == world * PER_RANK and int(bad) == 0
        assert int(first) == r * PER_RANK
    # the shards concatenated equal the single-process derivation of the whole batch
    got = np.concatenate([np.load(tmp_path / f"ss_{r}.npy") for r in range(world)])
    coins = orc.bench_coins(world * PER_RANK, 96, SEED, 0)
    pk, _ = orc.batch_keypair(ALG, np.ascontiguousarray(coins[:, :64]))
    _, ss = orc.batch_encaps(ALG, pk, np.ascontiguousarray(coins[:, 64:]))
    assert np.array_equal(got, ss)


def test_shard_arithmetic():
    from qrkem.shard import strong_shard, weak_shard
    for world in (1, 2, 3, 8):
        tot = 1000
        parts = [strong_shard(r, world, tot) for r in range(world)]
        assert sum(p.count for p in parts) == tot
        assert all(parts[i].first + parts[i].count == parts[i + 1].first for i in range(world - 1))
        w = [weak_shard(r, world, 1 << 20) for r in range(world)]
        assert w[-1].first == (world - 1) << 20
    with pytest.raises(ValueError):
        weak_shard(2, 2, 10)
