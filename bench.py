#!/usr/bin/env python3
"""Bench: ML-KEM-768 encaps+decaps per second at batch 2^20 per GPU (BASELINE.json).

One step = batched Encaps over 2^20 device-resident public keys followed by
batched Decaps of the resulting ciphertexts (the reference's per-handshake
OQS_KEM_encaps + OQS_KEM_decaps pair, quantum_resistant_p2p/vendor/oqs.py:348,372,
times 2^20).  KeyGen runs once, untimed (reported as keygen_per_s).  Inputs are
derived on device from (seed, global index) so shards are identical whatever the
GPU count; ranks take contiguous index ranges (weak scaling, no data-path
collective; one all_reduce of counters + max elapsed at the end).

python bench.py [--gpus N --steps K --warmup W] [--alg ML-KEM-768] [--log2-batch 20]
                [--mode encdec|decaps-tampered] [--no-cpu]
For N > 1 launch with torch.distributed.run (one rank per GPU, RCCL backend).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT / "quantum-resistant-p2p_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

METRIC = "ML-KEM-768 encaps+decaps/sec (node) at batch 2^20, 1/2/4/8 GPU; % VALU peak"

# ---------------------------------------------------------------- work model (DESIGN.md "Roofline")
PERM_OPS = 4320  # VALU ops per Keccak-f[1600] on gfx950 (180 per round x 24, one lane)
# Peak int32 VALU lane-ops/s: 256 CU x 4 SIMD x 32 lanes x 2.4 GHz (MI355X_MICROARCH.md:
# 4 SIMD-32 per CU; 157.3 TF FP32 vector = this rate x 2 flop/FMA).
VALU_PEAK = 256 * 4 * 32 * 2.4e9
KP = {"ML-KEM-512": (2, 3, 2, 10, 4), "ML-KEM-768": (3, 2, 2, 10, 4), "ML-KEM-1024": (4, 2, 2, 11, 5)}


def mlkem_sizes(alg):
    k, _, _, du, dv = KP[alg]
    return 384 * k + 32, 768 * k + 96, 32 * (du * k + dv)


def perms_encdec(alg) -> int:
    """FIPS-minimal Keccak permutations per Encaps + Decaps (SampleNTT at 3 blocks)."""
    k, eta1, eta2, _, _ = KP[alg]
    pk, _, ct = mlkem_sizes(alg)
    h_ek = (pk + 1 + 135) // 136          # H(ek)      SHA3-256
    g = 1                                  # G(m || h)  SHA3-512
    prf = k * (1 if eta1 == 2 else 2) + (k + 1)
    xof = 3 * k * k
    j = (32 + ct + 1 + 135) // 136         # J(z || c)  SHAKE256
    enc = h_ek + g + prf + xof
    dec = g + prf + xof + j
    return enc + dec


def valu_ops_encdec(alg) -> int:
    """W = P*4320 + (NTT + NTT^-1)*896*8 + basemul_polys*3584."""
    k = KP[alg][0]
    ntts = (k + (k + 1)) + (k + 1) + (k + (k + 1))  # enc: k fwd, k+1 inv; dec: k fwd + 1 inv; re-enc
    basemul_polys = (k * k + k) + k + (k * k + k)
    return perms_encdec(alg) * PERM_OPS + ntts * 896 * 8 + basemul_polys * 3584


def kernel_ops_per_instance(alg, name):
    """Algorithmic VALU ops of one lane-instance of a Keccak-stage kernel (launch = instances x this)."""
    k, eta1, _, _, _ = KP[alg]
    pk, _, ct = mlkem_sizes(alg)
    if name == "k_xof":
        return 3 * PERM_OPS, k * k
    if name == "k_front_encaps":
        return ((pk + 1 + 135) // 136 + 1) * PERM_OPS, 1
    if name == "k_front_decaps":
        return (1 + (32 + ct + 1 + 135) // 136) * PERM_OPS, 1
    if name == "k_prf":
        return ((k * (1 if eta1 == 2 else 2) + (k + 1)) * PERM_OPS) / (2 * k + 1), 2 * k + 1
    return None, None


# ---------------------------------------------------------------- helpers
def env_int(name, default):
    v = os.environ.get(name)
    return int(v) if v not in (None, "") else default


def cpu_threads() -> int:
    n = os.cpu_count() or 1
    cap = env_int("OMP_NUM_THREADS", 16)
    return max(1, min(n, cap, 16))


def cpu_baseline(alg, pk, sk, ec, ct_gpu, ss_gpu, B):
    """Oracle (C restatement, 'port') timed on host cores over a bounded sample; also checks
    the GPU outputs for the sampled indices byte-for-byte."""
    sys.path.insert(0, str(ROOT / "oracle"))
    import oracle as orc
    threads = cpu_threads()

    def take(t, n):
        return np.ascontiguousarray(t[:n].cpu().numpy())

    cal = min(1024, B)
    pk_c, sk_c, ec_c = take(pk, cal), take(sk, cal), take(ec, cal)
    t0 = time.perf_counter()
    c, s = orc.batch_encaps(alg, pk_c, ec_c, threads)
    orc.batch_decaps(alg, sk_c, c, threads)
    rate = cal / max(time.perf_counter() - t0, 1e-6)
    S = int(min(B, max(cal, (rate * 12.0) // 1024 * 1024)))
    pk_s, sk_s, ec_s = take(pk, S), take(sk, S), take(ec, S)
    t0 = time.perf_counter()
    c, s = orc.batch_encaps(alg, pk_s, ec_s, threads)
    s2 = orc.batch_decaps(alg, sk_s, c, threads)
    dt = time.perf_counter() - t0
    match = bool(np.array_equal(c, take(ct_gpu, S)) and np.array_equal(s, take(ss_gpu, S))
                 and np.array_equal(s2, s))
    # the reference call pattern: one handshake per Python call, one core
    t0 = time.perf_counter()
    m = 0
    while time.perf_counter() - t0 < 2.0 and m < S:
        cc, ss_ = orc.encaps(alg, pk_s[m].tobytes(), ec_s[m].tobytes())
        orc.decaps(alg, sk_s[m].tobytes(), cc)
        m += 1
    single = m / (time.perf_counter() - t0)
    return {
        "value": S / dt, "unit": "handshakes/s", "cores": threads, "kind": "port",
        "sample": f"first {S} handshakes of the same workload (oracle/liboracle.so, C restatement of "
                  f"FIPS 203, -O3 -march=native, {threads} pthreads); liboqs itself is absent "
                  f"(.MISSING_LARGE_BLOBS:1)",
        "sample_matches_gpu": match,
        "single_core_python_per_call": single,
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--alg", default="ML-KEM-768")
    ap.add_argument("--log2-batch", type=int, default=20)
    ap.add_argument("--chunk", type=int, default=1 << 20)
    ap.add_argument("--seed", type=lambda x: int(x, 0), default=0x5EED)
    ap.add_argument("--mode", choices=["encdec", "decaps-tampered"], default="encdec")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-profile", action="store_true")
    args = ap.parse_args()

    world = env_int("WORLD_SIZE", 1)
    rank = env_int("RANK", 0)
    local = env_int("LOCAL_RANK", 0)
    if world != args.gpus and rank == 0:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE {world}", file=sys.stderr)
    torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    from qrkem.batch import BatchKEM
    alg = args.alg
    B = 1 << args.log2_batch
    eng = BatchKEM(alg, device=local, chunk=args.chunk)
    from qrkem.shard import reduce_run, weak_shard
    base = weak_shard(rank, world, B).first  # global index range [base, base + B)

    coins = eng.bench_coins(B, 96, args.seed, base)
    kc = coins[:, :64].contiguous()
    ec = coins[:, 64:].contiguous()
    del coins
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    pk, sk = eng.keypair(coins=kc)
    torch.cuda.synchronize()
    keygen_s = time.perf_counter() - t0

    def barrier():
        if world > 1:
            dist.barrier()

    if args.mode == "encdec":
        def step():
            ct_, ss_ = eng.encaps(pk, coins=ec)
            ss2_ = eng.decaps(sk, ct_)
            return ct_, ss_, ss2_
    else:
        ct0, ss0 = eng.encaps(pk, coins=ec)
        eng.tamper(ct0, args.seed, 2)

        def step():
            return ct0, ss0, eng.decaps(sk, ct0)

    for _ in range(args.warmup):
        out = step()
    torch.cuda.synchronize()
    if not args.no_profile:
        eng.profile(True)
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        out = step()
    torch.cuda.synchronize()
    barrier()
    elapsed = time.perf_counter() - t0
    prof_live = eng.profile_read() if not args.no_profile else {}
    eng.profile(False)
    # Kernel-in-isolation pass (serial schedule, one untimed step): the forked
    # schedule overlaps kernel chains, which inflates per-kernel event durations.
    prof = {}
    if not args.no_profile:
        eng.set_streams(1)
        eng.profile(True)
        step()
        torch.cuda.synchronize()
        prof = {k: (ms, cnt) for k, (ms, cnt) in eng.profile_read().items()}
        eng.profile(False)
        eng.set_streams(2)

    ct, ss, ss2 = out
    mismatches = int((ss != ss2).any(dim=1).sum().item()) if args.mode == "encdec" else 0
    elapsed, (mismatches,) = reduce_run(elapsed, [mismatches], device=f"cuda:{local}")

    total = B * world * args.steps
    value = total / elapsed
    ms_per_step = elapsed * 1e3 / args.steps

    # ---------------- roofline of the dominant kernel (live HIP events on the launch stream)
    roof = None
    kernels = {}
    for name, (ms, cnt) in prof.items():
        kernels[name] = {"avg_ms": ms / cnt, "launches": cnt, "share": None}
    tot_ms = sum(ms for ms, _ in prof.values()) or 1.0
    for name, (ms, _) in prof.items():
        kernels[name]["share"] = ms / tot_ms
    if prof:
        dom = max(prof, key=lambda k: prof[k][0])
        per_inst, inst_per_hs = kernel_ops_per_instance(alg, dom)
        ms, cnt = prof[dom]
        chunk = min(args.chunk, B)
        if per_inst is not None:
            ops_per_launch = per_inst * inst_per_hs * chunk
            achieved = ops_per_launch / (ms / cnt * 1e-3)
            roof = {"kernel": dom, "bound": "valu", "achieved": achieved / 1e12, "peak": VALU_PEAK / 1e12,
                    "unit": "Top/s (int32 lane-ops)", "frac": achieved / VALU_PEAK, "traffic": None,
                    "ops_per_launch": ops_per_launch, "avg_launch_ms": ms / cnt}

    W = valu_ops_encdec(alg) if args.mode == "encdec" else None
    result = {
        "metric": METRIC if (alg == "ML-KEM-768" and args.mode == "encdec")
        else f"{alg} {args.mode} /sec at batch 2^{args.log2_batch} per GPU",
        "value": value,
        "unit": "encaps+decaps/s" if args.mode == "encdec" else "decaps/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_per_step,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u32",
        "data": "synthetic: coins = SHAKE256('qrk-bench'||LE64(seed)||LE64(i)) generated on device; "
                "keys from batched KeyGen on those coins",
        "config": {"workload": f"{alg} {'Encaps+Decaps' if args.mode == 'encdec' else 'Decaps, 50% tampered'}"
                               f" of 2^{args.log2_batch} device-resident handshakes per GPU (BASELINE.json configs[1])",
                   "alg": alg, "batch_per_gpu": B, "global_batch": B * world, "chunk": min(args.chunk, B),
                   "parallelism": f"index-sharded x{world} (no data-path collective)"},
        "roofline": roof,
        "valu_frac_of_peak_step": (value * W / VALU_PEAK) if W else None,
        "valu_ops_per_handshake": W,
        "keygen_per_s": B * world / keygen_s if keygen_s > 0 else None,
        "kernels": kernels,
        "kernels_timed_region_forked": {k: {"avg_ms": ms / c, "launches": c} for k, (ms, c) in prof_live.items()},
        "checks": {"ss_enc_eq_ss_dec_mismatches": mismatches if args.mode == "encdec" else None},
        "cpu_baseline": None,
    }
    if rank == 0 and world == 1 and not args.no_cpu and args.mode == "encdec":
        result["cpu_baseline"] = cpu_baseline(alg, pk, sk, ec, ct, ss, B)
    if rank == 0:
        print(json.dumps(result))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
