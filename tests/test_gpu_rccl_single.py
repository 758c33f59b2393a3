"""The RCCL ("nccl") calls of the multi-GPU bench path, on the one GPU a test box has.

`bench.py --gpus N` runs one rank per GPU: `init_process_group("nccl", device_id=cuda:local)`,
then `qrkem.shard.reduce_run` (all_reduce MAX of a float64 and SUM of int64 counters on the GPU)
and `gather_digests` (all_gather_object).  Two ranks cannot share one GPU under RCCL, so this runs
the same calls in a world of one rank -- RCCL initialised on the device, the same dtypes, ops and
object gather -- with the world-size shortcut of `reduce_run` / `gather_digests` bypassed.  The
multi-rank logic itself is covered on the CPU with gloo (`test_multirank_gloo.py`).
"""
import os
import socket
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]

SCRIPT = r"""
import sys, torch, torch.distributed as dist
sys.path.insert(0, sys.argv[1])
from qrkem import shard
torch.cuda.set_device(0)
dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{sys.argv[2]}", rank=0, world_size=1,
                        device_id=torch.device("cuda", 0))
assert dist.get_backend() == "nccl"
# reduce_run's body with the world-size shortcut bypassed
t = torch.tensor([1.25], dtype=torch.float64, device="cuda:0")
c = torch.tensor([3, 1 << 40, 7], dtype=torch.int64, device="cuda:0")
dist.all_reduce(t, op=dist.ReduceOp.MAX)
dist.all_reduce(c, op=dist.ReduceOp.SUM)
assert float(t.item()) == 1.25 and c.tolist() == [3, 1 << 40, 7]
# gather_digests' body
parts = [None]
dist.all_gather_object(parts, {0: "ab", 1: "cd"})
assert parts == [{0: "ab", 1: "cd"}]
dist.barrier()
# the functions themselves (identity at world size 1)
assert shard.reduce_run(2.5, [4, 5], device="cuda:0") == (2.5, [4, 5])
assert shard.gather_digests({3: "ef"}) == {3: "ef"}
torch.cuda.synchronize()
dist.destroy_process_group()
print("rccl ok")
"""


@pytest.mark.gpu
def test_rccl_calls_of_the_bench_path():
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    p = subprocess.run([sys.executable, "-c", SCRIPT, str(ROOT / "quantum-resistant-p2p_amd"), str(port)],
                       env=env, capture_output=True, text=True, timeout=110)
    assert p.returncode == 0, p.stderr[-3000:]
    assert "rccl ok" in p.stdout
