"""GPU, world size 2 (gloo for the end-of-run collectives): two ranks, each with its own
libqrkem context on cuda:0, run the sharded path exactly as `bench.py` does -- coins
from (seed, global index) through qrk_bench_coins with the rank's `first` offset,
KeyGen / Encaps / Decaps, per-record digests -- then reduce counters / max elapsed with
reduce_run and gather the block digests.  The union must equal one process doing the
whole batch, and the reduced counters must add up.  (The CPU variant in
test_multirank_gloo.py runs the oracle per rank; this one drives the HIP path.)
"""
import os
import socket

import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu

ALG = "ML-KEM-768"
TOTAL = 1 << 14
BLOCK = 1 << 12
SEED = 0x5EED


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _shard(eng, first, count):
    coins = eng.bench_coins(count, 96, SEED, first)
    kc, ec = coins[:, :64].contiguous(), coins[:, 64:].contiguous()
    pk, sk = eng.keypair(coins=kc)
    ct, ss = eng.encaps(pk, coins=ec)
    ss2 = eng.decaps(sk, ct)
    rec = eng.digest_rows(ct, ss)
    torch.cuda.synchronize()
    return int((ss != ss2).any(dim=1).sum().item()), rec.cpu().numpy()


def _worker(rank, world, port, outdir):
    import json
    import sys
    from pathlib import Path
    root = Path(__file__).resolve().parents[1]
    sys.path[:0] = [str(root / "quantum-resistant-p2p_amd")]
    import torch.distributed as dist
    from qrkem.batch import BatchKEM
    from qrkem.shard import block_digests, gather_digests, reduce_run, strong_shard
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    sh = strong_shard(rank, world, TOTAL)
    eng = BatchKEM(ALG, device=0)
    bad, rec = _shard(eng, sh.first, sh.count)
    elapsed, (done, bad) = reduce_run(1.0 + rank, [sh.count, bad])
    blocks = gather_digests(block_digests(rec, sh.first, BLOCK))
    with open(os.path.join(outdir, f"r{rank}.json"), "w") as f:
        json.dump({"elapsed": elapsed, "done": done, "bad": bad, "blocks": blocks, "first": sh.first}, f)
    dist.barrier()
    dist.destroy_process_group()
    eng.close()


def test_two_ranks_drive_batchkem_and_match_one_process(tmp_path):
    import json

    import torch.multiprocessing as mp
    from qrkem.batch import BatchKEM
    from qrkem.shard import block_digests
    world = 2
    mp.start_processes(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True,
                       start_method="spawn")
    res = [json.load(open(tmp_path / f"r{r}.json")) for r in range(world)]
    eng = BatchKEM(ALG, device=0)
    bad, rec = _shard(eng, 0, TOTAL)
    want = {str(k): v for k, v in block_digests(rec, 0, BLOCK).items()}
    assert bad == 0
    for r, d in enumerate(res):
        assert d["elapsed"] == 1.0 + (world - 1)  # max over ranks
        assert d["done"] == TOTAL and d["bad"] == 0
        assert d["first"] == r * TOTAL // world
        assert d["blocks"] == want  # every rank holds the gathered union
