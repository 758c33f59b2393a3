"""CPU: bench.py's own multi-rank launcher (`python bench.py --gpus N` without torchrun) and the
strong-scaling digest block choice.  The launcher must start the N ranks as a child process
(never exec, no HIP call in the parent) on 127.0.0.1 and relay rank 0's single JSON line."""
import json
import os
import sys
import textwrap
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "quantum-resistant-p2p_amd"))

bench = pytest.importorskip("bench")


def test_launcher_argv_and_env():
    argv = bench.launcher_argv(["--gpus", "8", "--steps", "3"], 8, 29511)
    assert argv[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=8" in argv and "--master-addr=127.0.0.1" in argv and "--master-port=29511" in argv
    assert argv[-4:] == ["--gpus", "8", "--steps", "3"]
    assert argv[-5].endswith("bench.py")
    env = bench.launcher_env({"RANK": "3", "WORLD_SIZE": "4", "MASTER_PORT": "1", "PATH": "/bin"})
    assert "RANK" not in env and "WORLD_SIZE" not in env and "MASTER_PORT" not in env
    assert env["PATH"] == "/bin" and env["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"
    assert bench.launcher_env({"HSA_ENABLE_IPC_MODE_LEGACY": "0"})["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"


def test_pick_json_line():
    text = 'noise\n{"metric": "m", "value": 1}\n{"not": "it"}\nmore\n'
    assert json.loads(bench.pick_json_line(text)) == {"metric": "m", "value": 1}
    assert bench.pick_json_line("nothing here\n{bad json") is None


def test_launch_ranks_runs_children_and_relays_rank0(tmp_path, capsys):
    """A stub rank script under the real torch.distributed.run: two ranks on gloo, rank 0 prints
    the line; the parent relays exactly that line."""
    stub = tmp_path / "stub.py"
    stub.write_text(textwrap.dedent('''
        import json, os, sys
        import torch.distributed as dist
        dist.init_process_group("gloo")
        r, w = dist.get_rank(), dist.get_world_size()
        dist.barrier()
        if r == 0:
            print("log line from rank 0")
            print(json.dumps({"metric": "stub", "value": w, "n_gpus": w, "argv": sys.argv[1:]}))
        dist.destroy_process_group()
    '''))
    rc = bench.launch_ranks(2, ["--gpus", "2", "--steps", "1"], script=stub)
    assert rc == 0
    out = capsys.readouterr().out.strip().splitlines()
    assert len(out) == 1
    d = json.loads(out[0])
    assert d["n_gpus"] == 2 and d["argv"] == ["--gpus", "2", "--steps", "1"]


@pytest.mark.parametrize("fail", [True, False])
def test_bench_module_exit_code_follows_the_ranks(tmp_path, fail):
    """`python bench.py --gpus 2` (the driver's multi-GPU invocation) exits non-zero when a rank
    fails, and 0 when rank 0 prints its line (the launcher's code was dropped)."""
    import subprocess
    stub = tmp_path / "stub.py"
    stub.write_text(textwrap.dedent(f'''
        import json, os, sys
        import torch.distributed as dist
        dist.init_process_group("gloo")
        r = dist.get_rank()
        dist.barrier()
        if r == 0 and not {fail}:
            print(json.dumps({{"metric": "stub", "value": 1}}))
        dist.destroy_process_group()
        sys.exit(3 if {fail} and r == 1 else 0)
    '''))
    env = dict(os.environ, QRK_BENCH_RANK_SCRIPT=str(stub))
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    p = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", "2", "--steps", "1"], env=env,
                       capture_output=True, text=True, timeout=300)
    if fail:
        assert p.returncode != 0, p.stdout + p.stderr
    else:
        assert p.returncode == 0, p.stdout + p.stderr
        assert json.loads(p.stdout.strip().splitlines()[-1])["metric"] == "stub"


@pytest.mark.parametrize("world,G,block", [(1, 24, 1 << 20), (2, 24, 1 << 20), (8, 24, 1 << 20), (16, 24, 1 << 20),
                                           (8, 22, 1 << 19), (4, 14, 1 << 12), (8, 14, None), (3, 24, None),
                                           (6, 24, None)])
def test_strong_digest_block(world, G, block):
    from qrkem.shard import block_digests, strong_shard
    assert bench.strong_digest_block(world, 1 << G) == block
    if block is not None:  # every rank's shard is aligned, so block_digests never raises
        import numpy as np
        for r in range(world):
            sh = strong_shard(r, world, 1 << G)
            if sh.count <= (1 << 16):
                block_digests(np.zeros((sh.count, 32), np.uint8), sh.first, block)
