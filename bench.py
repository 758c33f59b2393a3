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
For N > 1 bench.py either runs under torch.distributed.run (one rank per GPU, RCCL backend) or,
started directly with --gpus N, launches the N ranks itself as a child process and relays rank 0's
line.
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
VALU_FULL_RATE = 61.26  # T lane-ops/s: measured v_xor_b32 issue ceiling (profiles/r1/valu_peak_r1b.json)
KP = {"ML-KEM-512": (2, 3, 2, 10, 4), "ML-KEM-768": (3, 2, 2, 10, 4), "ML-KEM-1024": (4, 2, 2, 11, 5)}


def mlkem_sizes(alg):
    k, _, _, du, dv = KP[alg]
    return 384 * k + 32, 768 * k + 96, 32 * (du * k + dv)


def mlkem_perms(alg):
    """FIPS-minimal Keccak permutations per Encaps and per Decaps (SampleNTT at 3 blocks)."""
    k, eta1, eta2, _, _ = KP[alg]
    pk, _, ct = mlkem_sizes(alg)
    h_ek = (pk + 1 + 135) // 136          # H(ek)      SHA3-256
    g = 1                                  # G(m || h)  SHA3-512
    prf = k * (1 if eta1 == 2 else 2) + (k + 1)
    xof = 3 * k * k
    j = (32 + ct + 1 + 135) // 136         # J(z || c)  SHAKE256
    return h_ek + g + prf + xof, g + prf + xof + j


def perms_encdec(alg) -> int:
    enc, dec = mlkem_perms(alg)
    return enc + dec


def valu_ops(alg, mode="encdec") -> int:
    """W = P*4320 + (NTT + NTT^-1)*896*8 + basemul_polys*3584 per Encaps+Decaps
    (mode "encdec") or per Decaps (mode "decaps-tampered").  FrodoKEM: P*4320 (the S'A
    contraction runs on MFMA and is priced separately)."""
    if alg in HQ:
        names = ["k_hqc_enc_expand", "k_hqc_enc_mul", "k_hqc_hash", "k_hqc_dec_expand", "k_hqc_decode"]
        return sum(kernel_ops_per_hs(alg, nm, mode)[0] for nm in names)
    if alg in FP:
        p = frodo_perms(alg)
        enc = p["k_fr_front_enc"] + p["k_fr_gen_at"] + p["k_fr_se_stream"] + p["k_fr_ss"]
        dec = p["k_fr_g2_dec"] + p["k_fr_gen_at"] + p["k_fr_se_stream"] + p["k_fr_ss"]
        return (enc + dec if mode == "encdec" else dec) * PERM_OPS
    k = KP[alg][0]
    enc_p, dec_p = mlkem_perms(alg)
    enc = enc_p * PERM_OPS + (k + (k + 1)) * 896 * 8 + (k * k + k) * 3584
    dec = dec_p * PERM_OPS + ((k + 1) + (k + (k + 1))) * 896 * 8 + (k + (k * k + k)) * 3584
    return enc + dec if mode == "encdec" else dec


def valu_ops_encdec(alg) -> int:
    return valu_ops(alg, "encdec")


# FrodoKEM (n, logq, sec, hash rate bytes): FrodoKEM spec round 3 / SURVEY.md 8a A18-A21
FP = {"FrodoKEM-640-SHAKE": (640, 15, 16, 168), "FrodoKEM-976-SHAKE": (976, 16, 24, 136),
      "FrodoKEM-1344-SHAKE": (1344, 16, 32, 136), "FrodoKEM-640-AES": (640, 15, 16, 168),
      "FrodoKEM-976-AES": (976, 16, 24, 136), "FrodoKEM-1344-AES": (1344, 16, 32, 136)}
# AES Gen(A): T-table AES-128 lookups the kernel performs per 16-byte block -- rounds 3-10 (8 x 16);
# the plaintext is zero except LE16(i) || LE16(j), so rounds 1-2 fold into per-handshake and
# per-row precompute (aes.cuh) and are not counted (the FIPS-minimal 160 overstated
# the rate by 1.25x).  One ds_read_b32 wave instruction takes 2 LDS cycles (MI355X_MICROARCH.md
# LDS table) -> 32 lookups per clock per CU
AES_LOOKUPS_PER_BLOCK = 128
LDS_LOOKUP_PEAK = 256 * 32 * 2.4e9
MFMA_I8_PEAK = 5.0e15  # dense int8 MFMA ops/s (MI355X_MICROARCH.md: I8 = 2x BF16 per clock, BF16 ~2.5 PF dense)


def frodo_sizes(alg):
    n, logq, sec, _ = FP[alg]
    pk = 16 + logq * n
    return pk, sec + pk + 16 * n + sec, logq * n + 8 * logq


def frodo_perms(alg):
    """Keccak permutations per Encaps / per Decaps, by kernel (FIPS-minimal sponge counts)."""
    n, logq, sec, rate = FP[alg]
    pk, _, ct = frodo_sizes(alg)
    se_words = (2 * n + 8) * 8 * 2 // 8
    gen_a = 0 if alg.endswith("-AES") else n * -(-2 * n // 168)  # SHAKE128 rows of A
    se = -(-se_words * 8 // rate)                      # SHAKE(0x96 || seedSE) stream
    ss = -(-(ct + sec + 1) // rate)                    # ss = H(ct || k)
    return {"k_fr_gen_at": gen_a, "k_fr_se_stream": se, "k_fr_ss": ss,
            "k_fr_front_enc": -(-(pk + 1) // rate) + 1, "k_fr_g2_dec": 1}


# HQC (n, n1, n2, w, w_r, w_e, k): the 2023-04-30 HQC parameter sets (oracle/py/hqc_spec.py)
HQ = {"HQC-128": (17669, 46, 384, 66, 75, 75, 16), "HQC-192": (35851, 56, 640, 100, 114, 114, 24),
      "HQC-256": (57637, 90, 640, 131, 149, 149, 32)}
# sparse-dense product in F2[X]/(X^n-1): one funnel shift + one XOR per (position, 32-bit word), and
# the word's window read from LDS.  Per wave and position (64 output words): the reads are >= 64
# dwords = 2 LDS clocks of the CU (128 B/clk), the VALU work one half-rate v_alignbit (4 SIMD clocks)
# + one v_xor (2) = 1.5 CU clocks over its 4 SIMDs -- so the products are priced against the LDS
# (LDS_LOOKUP_PEAK, one ds_read_b32 lane per word and position), with the VALU view kept beside it
# (`valu_frac`).  The kernels read (WPT + 1) / WPT window words per output word (1.2 at WPT = 5).
SPARSE_OPS = 2


def hqc_work(alg):
    """Per-call algorithmic work of each HQC kernel: Keccak permutations (FIPS-minimal sponge
    counts, 17-word SHAKE256 blocks) or sparse-dense word operations."""
    n, n1, n2, w, wr, we, k = HQ[alg]
    nb, vb = (n + 7) // 8, n1 * n2 // 8
    nw32, vw32 = (n + 31) // 32, vb // 4
    rw = lambda x: (4 * x + 7) // 8  # noqa: E731  seedexpander words of a weight-x vector
    blocks = lambda words: -(-words // 17)  # noqa: E731
    mw = (k + nb + vb + 2 + 7) // 8
    return {"perms": {"k_hqc_enc_expand": 1 + blocks(2 * rw(wr) + rw(we)) + blocks((nb + 7) // 8),
                      "k_hqc_dec_expand": blocks(2 * rw(w)), "k_hqc_hash": blocks(mw),
                      "k_hqc_kg_expand": blocks(2 * rw(w)) + blocks((nb + 7) // 8)},
            "ops": {"k_hqc_enc_mul": 2 * wr * nw32 * SPARSE_OPS, "k_hqc_decode": w * vw32 * SPARSE_OPS,
                    "k_hqc_kg_mul": w * nw32 * SPARSE_OPS}}


# ML-KEM polynomial cores: per-stage lane-instruction counts of the minimal gfx950 sequence for
# each stage as the cores implement it (DESIGN.md "Pricing the polynomial cores"); FIPS 203
# Alg. 9-12 plus CBD, compress and the byte codecs.
FWD_NTT = 7 * 128 * 6              # fp32 butterfly: v_mul, v_fmamk, v_sub (magic), v_fma, v_add, v_sub
INV_NTT = 7 * 128 * 6 + 2 * 128 * 3 + 256 * 4  # + the two reduced sum layers + the 128^-1 scaling modmul
NTT_MIDRED = 256 * 3               # decrypt: inputs up to q, one reduction after layer 4
CBD_OPS = {2: 256 * 3, 3: 256 * 4}  # SWAR nibble sums + fp32 conversion per coefficient
BOP = 128 * 10                     # basemul operand (b0, b1*gamma) / (b1, b0) from an NTT output
BMUL = 128 * 2                     # one (row, j) term: two v_dot2c_i32_i16 per coefficient pair
ACC = 256 * 8                      # int32 accumulator -> centered fp32 residue (acc_to_f)
COMPRESS = 256 * 6                 # canonicalise + Compress_d (mulhi) per coefficient
DEC12 = 256 * 2                    # ByteDecode_12 + the FIPS 203 7.2 modulus reduction
ENC12 = 256 * 3                    # canonicalise + ByteEncode_12
UNPACK = 256 * 4                   # ByteDecode_d + Decompress_d per coefficient
PACK = 256 * 2                     # ByteEncode_d per coefficient
DEC_MSG = 256 * 6                  # Decaps: Decompress_dv(v) - w, canonicalise, Compress_1


def mlkem_core_ops(k, eta1, kind):
    """Algorithmic lane-ops per handshake of one launch of an ML-KEM polynomial core."""
    if kind == "encrypt":  # K-PKE.Encrypt (Encaps, and the Decaps re-encryption)
        return (k * CBD_OPS[eta1] + (k + 1) * CBD_OPS[2] + k * FWD_NTT + k * BOP + (k * k + k) * BMUL
                + (k + 1) * (ACC + INV_NTT + COMPRESS + PACK) + k * DEC12)
    if kind == "decrypt":  # K-PKE.Decrypt
        return (k + 1) * UNPACK + k * (FWD_NTT + NTT_MIDRED + DEC12 + BOP + BMUL) + ACC + INV_NTT + DEC_MSG
    if kind == "keygen":   # K-PKE.KeyGen: s, e sampling + NTT, t = A s + e, both encodings
        return 2 * k * (CBD_OPS[eta1] + FWD_NTT) + k * BOP + k * k * BMUL + k * ACC + 3 * k * ENC12
    raise ValueError(kind)


ONE_OP_KERNELS = {"k_front_encaps", "k_j_decaps", "k_g_decaps", "k_decrypt_core", "k_front_decaps"}


def kernel_ops_per_hs(alg, name, mode, calls=None):
    """Algorithmic ops one handshake contributes to kernel `name` in one bench step
    (encaps+decaps, or decaps only) and the bound they are priced against.  A multi-role launch
    ("k_front_encaps+k_xof", mlkem.hip k_multi) carries the sum of its roles' ops (the SampleNTT
    fix-up, ~0.7 % of the entries, is not counted); it runs once per step when one of its roles
    belongs to Encaps or Decaps alone, so its shared roles (SampleNTT, PRFs) count once then.
    `calls` overrides how many of the step's operations run a shared kernel."""
    if "+" in name:
        roles = name.split("+")
        c = 1 if any(r in ONE_OP_KERNELS for r in roles) else None
        parts = [kernel_ops_per_hs(alg, r, mode, c) for r in roles]
        ops = [o for o, _ in parts if o is not None]
        bounds = {b for o, b in parts if o is not None}
        if not ops:
            return None, None
        return sum(ops), (bounds.pop() if len(bounds) == 1 else "valu")
    if calls is None:
        calls = 2 if mode == "encdec" else 1  # kernels shared by Encaps and Decaps run once per op
    if alg in HQ:
        wk = hqc_work(alg)
        once = name in ("k_hqc_dec_expand", "k_hqc_decode")  # Decaps-only kernels
        c = 1 if once else calls
        if name in wk["perms"]:
            return c * wk["perms"][name] * PERM_OPS, "valu"
        if name in wk["ops"]:
            return c * wk["ops"][name] // SPARSE_OPS, "lds"  # LDS word reads (see SPARSE_OPS)
        return None, None
    if alg in FP:
        n = FP[alg][0]
        perms = frodo_perms(alg)
        if name == "k_fr_gen_mm":  # Gen(A) Keccak (the bound) fused with S'A on MFMA
            return calls * perms["k_fr_gen_at"] * PERM_OPS, "valu"
        if name in ("k_fr_gen_mm_aes", "k_fr_gen_mv_aes"):
            # Gen(A) AES-128 T-table lookups (LDS) fused with S'A (on MFMA, or column-major on VALU
            # in k_fr_gen_mv_aes): the same n * n/8 blocks either way
            return calls * n * (n // 8) * AES_LOOKUPS_PER_BLOCK, "lds"
        if name in ("k_fr_front_enc",):
            return (perms[name] * PERM_OPS if mode == "encdec" else None), "valu"
        if name in perms:
            return calls * perms[name] * PERM_OPS, "valu"
        return None, None
    k, eta1, _, _, _ = KP[alg]
    pk, _, ct = mlkem_sizes(alg)
    if name == "k_xof":
        return calls * 3 * k * k * PERM_OPS, "valu"
    if name == "k_front_encaps" and mode == "encdec":
        return ((pk + 1 + 135) // 136 + 1) * PERM_OPS, "valu"
    if name == "k_front_decaps":  # G(m' || h) + J(z || c) (rounds 1-3: one kernel)
        return (1 + (32 + ct + 1 + 135) // 136) * PERM_OPS, "valu"
    if name == "k_j_decaps":  # J(z || c)
        return ((32 + ct + 1 + 135) // 136) * PERM_OPS, "valu"
    if name == "k_g_decaps":  # G(m' || h)
        return PERM_OPS, "valu"
    if name == "k_prf":
        return calls * (k * (1 if eta1 == 2 else 2) + (k + 1)) * PERM_OPS, "valu"
    if name == "k_encrypt_core":  # Encaps' Encrypt, and Decaps' re-encryption
        return calls * mlkem_core_ops(k, eta1, "encrypt"), "valu"
    if name == "k_decrypt_core":
        return mlkem_core_ops(k, eta1, "decrypt"), "valu"
    if name == "k_keygen_core":
        return mlkem_core_ops(k, eta1, "keygen"), "valu"
    return None, None


def survey_core_ops(alg, name, mode):
    """SURVEY.md 8d's W terms for an ML-KEM polynomial core, per handshake and step: 896 x 8 ops
    per NTT or NTT^-1 and 3584 per basemul polynomial (sampling, packing and compare omitted),
    an independent pricing of the cores next to bench.py's own instruction model."""
    if alg not in KP:
        return None
    k = KP[alg][0]
    calls = 2 if mode == "encdec" else 1
    ntt, bm = 896 * 8, 3584
    if name == "k_encrypt_core":  # NTT(y_j), NTT^-1 of the k u-rows and v; A^T y and t^T y
        return calls * ((2 * k + 1) * ntt + (k * k + k) * bm)
    if name == "k_decrypt_core":  # NTT(u_j), NTT^-1(s^T u); s^T u
        return (k + 1) * ntt + k * bm
    if name == "k_keygen_core":  # NTT(s_j), NTT(e_i); A s
        return 2 * k * ntt + k * k * bm
    return None


RED_DEVICE = None  # device of the end-of-run reduction tensors (None = host, for gloo)


# ---------------------------------------------------------------- helpers
def env_int(name, default):
    v = os.environ.get(name)
    return int(v) if v not in (None, "") else default


def host_cpu() -> dict:
    """The host cores this job may use and the CPU model (SURVEY.md 8d CPU baseline (ii)).
    On the GPU box nproc / os.cpu_count() report the whole machine while the job's cgroup
    quota (cpu.max) allots it a share: the baseline uses every core of that share."""
    aff = len(os.sched_getaffinity(0))
    quota = None
    try:
        q, period = Path("/sys/fs/cgroup/cpu.max").read_text().split()
        if q != "max":
            quota = -(-int(q) // int(period))
    except (OSError, ValueError):
        pass
    model = None
    try:
        for line in Path("/proc/cpuinfo").read_text().splitlines():
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    cores = min(aff, quota) if quota else aff
    return {"cores": cores, "model": model, "logical_cpus_on_host": os.cpu_count(), "affinity_cpus": aff,
            "cgroup_quota_cores": quota}


def cpu_threads() -> int:
    return host_cpu()["cores"]


def cpu_baseline(alg, mode, kc, pk, sk, ec, ct_in, ss_gpu, B):
    """Oracle (C restatement, 'port') timed on every host core this job may use, over a bounded
    sample (~12 s); also checks the GPU outputs for the sampled indices byte-for-byte, KeyGen
    included (the sample's keys are regenerated on the CPU from the same coins).
    mode "encdec": Encaps(pk, ec) + Decaps; ct_in / ss_gpu = the GPU's ct / ss.
    mode "decaps-tampered": Decaps(sk, ct_in) only; ss_gpu = the GPU's ss."""
    sys.path.insert(0, str(ROOT / "oracle"))
    import oracle as orc
    cpu = host_cpu()
    threads = cpu["cores"]

    def take(t, n):
        return np.ascontiguousarray(t[:n].cpu().numpy())

    def run(n, opk, osk):
        if mode == "encdec":
            c, s = orc.batch_encaps(alg, opk[:n], take(ec, n), threads)
            return c, s, orc.batch_decaps(alg, osk[:n], c, threads, with_status=True)[0]
        return None, None, orc.batch_decaps(alg, osk[:n], take(ct_in, n), threads, with_status=True)[0]

    cal = min(256 if (alg in FP or alg in HQ) else 1024, B)
    opk, osk = orc.batch_keypair(alg, take(kc, cal), threads)
    t0 = time.perf_counter()
    run(cal, opk, osk)
    rate = cal / max(time.perf_counter() - t0, 1e-6)
    S = int(min(B, max(cal, (rate * 12.0) // 256 * 256)))
    # KeyGen of the sample on the CPU (untimed, as on the GPU): the GPU's keys must match
    t0 = time.perf_counter()
    opk, osk = orc.batch_keypair(alg, take(kc, S), threads)
    keygen_rate = S / max(time.perf_counter() - t0, 1e-6)
    keygen_match = bool(np.array_equal(opk, take(pk, S)) and np.array_equal(osk, take(sk, S)))
    t0 = time.perf_counter()
    c, s, s2 = run(S, opk, osk)
    dt = time.perf_counter() - t0
    if mode == "encdec":
        match = bool(np.array_equal(c, take(ct_in, S)) and np.array_equal(s, take(ss_gpu, S))
                     and np.array_equal(s2, s))
    else:
        match = bool(np.array_equal(s2, take(ss_gpu, S)))
    # the reference call pattern: one handshake per Python call, one core
    pk_s, ec_s, ct_s = opk, take(ec, S), take(ct_in, S)
    t0 = time.perf_counter()
    m = 0
    while time.perf_counter() - t0 < 2.0 and m < S:
        if mode == "encdec":
            cc, _ = orc.encaps(alg, pk_s[m].tobytes(), ec_s[m].tobytes())
        else:
            cc = ct_s[m].tobytes()
        orc.decaps_rc(alg, osk[m].tobytes(), cc)
        m += 1
    single = m / (time.perf_counter() - t0)
    # KeyGen one call at a time on one core: the protocol runs it twice per exchange
    # (messaging.py:590, 809; key_exchange.py:133)
    kc_s = take(kc, min(S, 4096))
    t0 = time.perf_counter()
    m_kg = 0
    while time.perf_counter() - t0 < 1.0 and m_kg < kc_s.shape[0]:
        orc.keypair(alg, kc_s[m_kg].tobytes())
        m_kg += 1
    single_kg = m_kg / (time.perf_counter() - t0)
    spec = "FrodoKEM round 3" if alg in FP else ("HQC 2023-04-30" if alg in HQ else "FIPS 203")
    return {
        "value": S / dt, "unit": "encaps+decaps/s" if mode == "encdec" else "decaps/s", "cores": threads,
        "kind": "port",
        "sample": f"first {S} handshakes of the same workload (oracle/liboracle.so, C restatement of "
                  f"{spec}, -O3 -march=native, {threads} pthreads = every core of this job's host share); "
                  f"liboqs itself is absent (.MISSING_LARGE_BLOBS:1)",
        "cpu": cpu,
        "sample_matches_gpu": match,
        "keygen_sample_matches_gpu": keygen_match,
        "keygen_per_s": keygen_rate,
        "single_core_python_per_call": single,
        "single_core_python_keygen_per_call": single_kg,
        "single_core_python_keygen_us_per_call": 1e6 / single_kg,
    }


def keccak_practical_peak():
    """Top/s (4320-op count) of a register-resident Keccak-f[1600] loop measured on MI355X: the
    best of tools/valu_peak.hip (profiles/r1/valu_peak_r1b.json) and tools/rot64_probe.hip's
    rounds-per-iteration variants (profiles/r2/rot64_unroll_probe.json, the kernels' two rounds
    per iteration), or None."""
    best = None
    for f in (ROOT / "profiles" / "r1" / "valu_peak_r1b.json", ROOT / "profiles" / "r2" / "rot64_unroll_probe.json"):
        try:
            d = json.loads(f.read_text())
            v = max(v for k, v in d.items() if k.startswith("keccak_") and k.endswith("_Tops_at_4320"))
            best = v if best is None or v > best else best
        except (OSError, ValueError):
            pass
    return best


def pmc_traffic(alg, mode, chunk, kernel):
    """HBM bytes per dispatch of `kernel` from the committed rocprofv3 PMC pass of the same
    configuration (profiles/pmc_traffic.json, written by tools/prof_summary.py), or None."""
    idx = ROOT / "profiles" / "pmc_traffic.json"
    if not idx.exists():
        return None, None
    e = json.loads(idx.read_text()).get(f"{alg}|{mode}|{chunk}")
    if not e:
        return None, None
    for k, v in e["hbm_bytes_per_dispatch"].items():
        if k == kernel or k.startswith(kernel + "<") and "true" not in k:
            return v, e["source"]
    return None, None


def pmc_issued(alg, mode, chunk, kernel):
    """Issued VALU lane-ops/s (T) of `kernel` in isolation from the committed SQ_INSTS_VALU pass
    of the same configuration (profiles/valu_rate.json, written by tools/valu_rate.py), or None."""
    idx = ROOT / "profiles" / "valu_rate.json"
    if not idx.exists():
        return None, None
    e = json.loads(idx.read_text()).get(f"{alg}|{mode}|{chunk}")
    if not e:
        return None, None
    for k, v in e["issued_Tops"].items():
        if k == kernel or k.startswith(kernel + "<") and "true" not in k:
            return v, e["source"]
    return None, None


def pmc_mfma(alg, mode, chunk, kernel):
    """Counter-derived MFMA utilisation of `kernel` from the committed rocprofv3 MFMA pass of the
    same configuration (profiles/mfma_util.json, written by tools/mfma_summary.py), or None."""
    idx = ROOT / "profiles" / "mfma_util.json"
    if not idx.exists():
        return None
    e = json.loads(idx.read_text()).get(f"{alg}|{mode}|{chunk}")
    if not e:
        return None
    for k, v in e["kernels"].items():
        if k == kernel or k.startswith(kernel + "<"):
            return {"mfma_util": v.get("mfma_util"), "mfma_i8_instrs_per_launch": v.get("mfma_i8_instrs_per_dispatch"),
                    "int8_ops_per_launch": v.get("int8_ops_per_dispatch"), "achieved_Tops": v.get("achieved_Tops"),
                    "frac": v.get("frac_of_int8_peak"), "source": e["source"],
                    "definition": "SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE x 1024 SIMDs); "
                                  "int8 ops = SQ_INSTS_VALU_MFMA_MOPS_I8 x 512 over the traced kernel time"}
    return None


def kernel_report(alg, mode, prof, B):
    """Per-kernel algorithmic rate: ops per handshake x B / total kernel time in `prof`
    (HIP-event durations).  Returns (kernels, roofline-of-dominant, mfma-object-or-None)."""
    kernels = {}
    tot_ms = sum(ms for ms, _ in prof.values()) or 1.0
    for name, (ms, cnt) in prof.items():
        ops, bound = kernel_ops_per_hs(alg, name, mode)
        kernels[name] = {"avg_ms": ms / cnt, "launches": cnt, "share": ms / tot_ms}
        if ops is not None:
            rate = ops * B / (ms * 1e-3)
            peak = {"mfma": MFMA_I8_PEAK, "lds": LDS_LOOKUP_PEAK}.get(bound, VALU_PEAK)
            kernels[name].update(bound=bound, achieved_Tops=rate / 1e12, frac=rate / peak)
            if alg in HQ and bound == "lds":  # the same product priced by its VALU ops
                kernels[name]["valu_frac"] = rate * SPARSE_OPS / VALU_PEAK
            sw = survey_core_ops(alg, name, mode)
            if sw is not None:  # the same kernel priced by SURVEY.md 8d's W (NTT + basemul terms only)
                kernels[name].update(survey_w_Tops=sw * B / (ms * 1e-3) / 1e12, survey_w_frac=sw * B / (ms * 1e-3) / peak)
    roof, mfma = None, None
    if prof:
        dom = max(prof, key=lambda k: prof[k][0])
        ops, bound = kernel_ops_per_hs(alg, dom, mode)
        ms, cnt = prof[dom]
        if ops is not None:
            achieved = ops * B / (ms * 1e-3)
            peak = {"mfma": MFMA_I8_PEAK, "lds": LDS_LOOKUP_PEAK}.get(bound, VALU_PEAK)
            roof = {"kernel": dom, "bound": bound, "achieved": achieved / 1e12, "peak": peak / 1e12,
                    "unit": {"valu": "Top/s (int32 lane-ops)", "lds": "T lookups/s (LDS ds_read_b32 lanes)"}.get(
                        bound, "Top/s (int8 MFMA ops)"),
                    "frac": achieved / peak, "traffic": None,
                    "ops_per_launch": ops * B / cnt, "avg_launch_ms": ms / cnt}
            if alg in HQ and bound == "lds":
                roof["valu_frac"] = achieved * SPARSE_OPS / VALU_PEAK
        gk = "k_fr_gen_mm_aes" if "k_fr_gen_mm_aes" in prof else "k_fr_gen_mm"
        if gk in prof:
            # S'A runs on MFMA inside the fused Gen(A) kernel: its rate is priced over that
            # kernel's whole duration (a lower bound on the MFMA pipe's own utilisation)
            n = FP[alg][0]
            calls = 2 if mode == "encdec" else 1
            ms, cnt = prof[gk]
            if gk == "k_fr_gen_mm_aes":
                tiles = n // 16
            else:
                tiles = sum(-(-min(84, n - 84 * b) // 16) for b in range(-(-2 * n // 168)))
            alg_ops = calls * 2 * 2 * 8 * n * n * B
            issued = calls * (-(-n // 64)) * tiles * 2 * (16 * 16 * 64 * 2) * B
            mfma = {"kernel": f"{gk} (S'A fused into Gen(A))", "achieved": alg_ops / (ms * 1e-3) / 1e12,
                    "issued": issued / (ms * 1e-3) / 1e12, "peak": MFMA_I8_PEAK / 1e12,
                    "unit": "Top/s (int8 MFMA ops; algorithmic = 2 limbs x 2 x 8 x n^2 per S'A)",
                    "frac": alg_ops / (ms * 1e-3) / MFMA_I8_PEAK, "avg_launch_ms": ms / cnt,
                    "note": "MFMA is not the bound: Gen(A) (Keccak or AES) is; see roofline"}
    return kernels, roof, mfma


# ---------------------------------------------------------------- handshake mode
SHA256_OPS = 1400  # VALU ops per SHA-256 compression (64 rounds x ~14 + 48-word schedule x ~10)


def hkdf_compressions(ikm_len, info_len, key_len):
    """HMAC-SHA256 extract + expand compressions for one key (hkdf.hip)."""
    blocks = lambda n: (n + 9 + 63) // 64  # noqa: E731
    extract = 1 + blocks(ikm_len) + 2
    nt = -(-key_len // 32)
    expand = 2 + sum(blocks((32 if r > 1 else 0) + info_len + 1) + 1 for r in range(1, nt + 1))
    return extract + expand


def mlkem_keygen_ops(alg):
    k, eta1, _, _, _ = KP[alg]
    pk, _, _ = mlkem_sizes(alg)
    perms = 1 + 2 * k * (1 if eta1 == 2 else 2) + 3 * k * k + (pk + 1 + 135) // 136
    return perms * PERM_OPS + 2 * k * 896 * 8 + k * k * 3584


def handshake_ops(alg, info_len, key_len):
    """Per handshake: 2 KeyGen + Encaps + Decaps + 2 HKDF (messaging.py:590, 809, 830, 845, 1038, 1068)."""
    return 2 * mlkem_keygen_ops(alg) + valu_ops(alg, "encdec") + \
        2 * hkdf_compressions(32, info_len, key_len) * SHA256_OPS


def node_uuid(tag: str, i: int) -> str:
    """UUID-formatted synthetic node id (the reference uses str(uuid.uuid4()),
    networking/node_identity.py:78)."""
    import hashlib
    h = hashlib.sha256(f"{tag}{i}".encode()).hexdigest()
    return f"{h[:8]}-{h[8:12]}-4{h[13:16]}-a{h[17:20]}-{h[20:32]}"


def bench_handshake(args, world, rank, local):
    """One step = N complete protocol key exchanges (qrk_handshake_batch) on device-resident
    coins and per-handshake HKDF infos; value = handshakes/s."""
    from qrkem.handshake import SYMMETRIC_KEY_SIZE, HandshakeDriver
    from qrkem.shard import reduce_run, weak_shard
    alg = args.alg
    frodo = alg in FP
    hqc = alg in HQ
    lb = args.log2_batch if args.log2_batch is not None else (16 if (frodo or hqc) else 20)
    B = 1 << lb
    drv = HandshakeDriver(alg, symmetric_name=args.symmetric, device=local, chunk=args.chunk)
    e = drv.engine
    base = weak_shard(rank, world, B).first
    kp, enc = e.kp_coins, e.enc_coins
    if 2 * kp <= 136:
        coins = e.bench_coins(B, 2 * kp, args.seed, base)  # KeyGen coins (initiator | responder)
        c_i, c_r = coins[:, :kp].contiguous(), coins[:, kp:].contiguous()
        del coins
    else:  # HQC: one SHAKE256 block per index and seed
        c_i = e.bench_coins(B, kp, args.seed, base)
        c_r = e.bench_coins(B, kp, args.seed ^ 0x5A5A, base)
    c_e = e.bench_coins(B, enc, args.seed ^ 0xE7C, base)  # Encaps coins: a second seed
    # peer p talks to this server node: infos differ per handshake (sorted ids, messaging.py:364-367)
    server = node_uuid("server-", rank)
    infos = [drv.info_for(node_uuid("peer-", base + i), server) for i in range(B)]
    info_len = sum(len(x) for x in infos) / B
    packed = drv.pack(infos)

    def step():
        return drv.run(packed, coins_kp_initiator=c_i, coins_kp_responder=c_r, coins_encaps=c_e)

    def barrier():
        if world > 1:
            dist.barrier()

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if not args.no_profile:
        e.profile(True)
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        out = step()
    torch.cuda.synchronize()
    barrier()
    elapsed = time.perf_counter() - t0
    prof = e.profile_read() if not args.no_profile else {}
    e.profile(False)
    disagree = int((out.agree != 1).sum().item())
    elapsed, (disagree,) = reduce_run(elapsed, [disagree], device=RED_DEVICE)
    value = B * world * args.steps / elapsed
    W = handshake_ops(alg, info_len, SYMMETRIC_KEY_SIZE[args.symmetric]) if not (frodo or hqc) else None
    kernels, roof = {}, None
    tot = sum(ms for ms, _ in prof.values()) or 1.0
    for name, (ms, cnt) in prof.items():
        kernels[name] = {"avg_ms": ms / cnt, "launches": cnt, "share": ms / tot}
    if "k_xof" in prof:  # the 2 KeyGen SampleNTT passes per handshake (Encaps' and Decaps' run
        k = KP[alg][0]      # inside multi-role launches, mlkem.hip k_multi)
        ms, cnt = prof["k_xof"]
        ops = 2 * 3 * k * k * PERM_OPS * B * args.steps
        roof = {"kernel": "k_xof", "bound": "valu", "achieved": ops / (ms * 1e-3) / 1e12,
                "peak": VALU_PEAK / 1e12, "unit": "Top/s (int32 lane-ops)",
                "frac": ops / (ms * 1e-3) / VALU_PEAK, "traffic": None, "avg_launch_ms": ms / cnt,
                "algorithmic_ops_per_launch": ops / cnt}
    result = {
        "metric": f"{alg} protocol handshakes/sec at batch 2^{lb} per GPU "
                  f"(2 KeyGen + Encaps + Decaps + 2 HKDF-SHA256)",
        "value": value, "unit": "handshakes/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": elapsed * 1e3 / args.steps, "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "u32",
        "data": "synthetic: coins = SHAKE256('qrk-bench'||LE64(seed)||LE64(i)) on device; UUID-formatted "
                "node ids, per-handshake HKDF info (messaging.py:364-367)",
        "config": {"workload": f"{alg} batched handshake driver, 2^{lb} exchanges per GPU (SURVEY.md 8f-1)",
                   "alg": alg, "symmetric": args.symmetric, "batch_per_gpu": B, "global_batch": B * world,
                   "mean_info_bytes": info_len, "parallelism": f"index-sharded x{world} (no data-path collective)"},
        "roofline": roof, "valu_frac_of_peak_step": value * W / (VALU_PEAK * world) if W else None, "valu_ops_per_unit": W,
        "kernels_timed_region": kernels, "checks": {"key_disagreements": disagree}, "cpu_baseline": None,
    }
    if rank == 0 and world == 1 and not args.no_cpu:
        sys.path.insert(0, str(ROOT / "oracle"))
        import oracle as orc
        threads = cpu_threads()
        take = lambda t, n: np.ascontiguousarray(t[:n].cpu().numpy())  # noqa: E731
        cal = min(B, 64 if (frodo or hqc) else 512)
        t0 = time.perf_counter()
        orc.batch_handshake(alg, take(c_i, cal), take(c_r, cal), take(c_e, cal), infos[:cal], drv.key_len, threads)
        rate = cal / (time.perf_counter() - t0)
        S = int(min(B, max(cal, (rate * 12.0) // 64 * 64)))
        t0 = time.perf_counter()
        pk_i, pk_r, c, key_i, key_r = orc.batch_handshake(alg, take(c_i, S), take(c_r, S), take(c_e, S), infos[:S],
                                                          drv.key_len, threads)
        dt = time.perf_counter() - t0
        match = all(np.array_equal(a, take(b, S)) for a, b in ((pk_i, out.pk_initiator), (pk_r, out.pk_responder),
                                                                (c, out.ciphertext), (key_i, out.key_initiator),
                                                                (key_r, out.key_responder)))
        result["cpu_baseline"] = {
            "value": S / dt, "unit": "handshakes/s", "cores": threads, "kind": "port", "cpu": host_cpu(),
            "sample": f"first {S} handshakes of the same workload (oracle/liboracle.so: "
                      f"{'FrodoKEM round 3' if frodo else ('HQC 2023-04-30' if hqc else 'FIPS 203')} + RFC 5869 C "
                      f"restatement, {threads} pthreads)",
            "sample_matches_gpu": match}
    if rank == 0:
        print(json.dumps(result))
    if world > 1:
        dist.destroy_process_group()


# ---------------------------------------------------------------- wire mode
HBM_PEAK = 8.0e12  # B/s, MI355X HBM3E (MI355X_MICROARCH.md)


def bench_wire(args, world, rank, local):
    """One step = the base64 work of B key exchanges: encode pk_i (messaging.py:607), decode it
    (:829), encode ct and pk_r (:852-853), decode ct (:1037).  value = handshakes/s."""
    from qrkem.shard import reduce_run
    from qrkem.wire import Base64Codec, encoded_len
    alg = args.alg
    if alg not in KP:
        raise SystemExit("wire mode: ML-KEM algorithms only in the bench")
    lb = args.log2_batch if args.log2_batch is not None else 20
    B = 1 << lb
    PK, _, CT = mlkem_sizes(alg)
    codec = Base64Codec(device=local)
    g = torch.Generator(device=f"cuda:{local}").manual_seed(args.seed + rank)
    pk_i = torch.randint(0, 256, (B, PK), dtype=torch.uint8, device=f"cuda:{local}", generator=g)
    pk_r = torch.randint(0, 256, (B, PK), dtype=torch.uint8, device=f"cuda:{local}", generator=g)
    ct_ = torch.randint(0, 256, (B, CT), dtype=torch.uint8, device=f"cuda:{local}", generator=g)

    def step():
        t_pk = codec.encode(pk_i)
        pk_rx, st1 = codec.decode(t_pk, PK)
        t_ct = codec.encode(ct_)
        t_pkr = codec.encode(pk_r)
        ct_rx, st2 = codec.decode(t_ct, CT)
        return t_pk, t_ct, t_pkr, pk_rx, ct_rx, st1, st2

    def barrier():
        if world > 1:
            dist.barrier()

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if not args.no_profile:
        _ctx_profile(codec, True)
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        out = step()
    torch.cuda.synchronize()
    barrier()
    elapsed = time.perf_counter() - t0
    prof = _ctx_profile_read(codec) if not args.no_profile else {}
    t_pk, t_ct, t_pkr, pk_rx, ct_rx, st1, st2 = out
    bad = int((pk_rx != pk_i).any(dim=1).sum().item() + (ct_rx != ct_).any(dim=1).sum().item()
              + st1.abs().sum().item() + st2.abs().sum().item())
    elapsed, (bad,) = reduce_run(elapsed, [bad], device=RED_DEVICE)
    value = B * world * args.steps / elapsed
    epk, ect = encoded_len(PK), encoded_len(CT)
    bytes_hs = 2 * (PK + epk) + (epk + PK + 4) + (CT + ect) + (ect + CT + 4)
    kernels, roof = {}, None
    per = {"k_b64_encode": 2 * (PK + epk) + (CT + ect), "k_b64_decode": (epk + PK + 4) + (ect + CT + 4)}
    for name, (ms, cnt) in prof.items():
        kernels[name] = {"avg_ms": ms / cnt, "launches": cnt}
        if name in per:
            rate = per[name] * B * args.steps / (ms * 1e-3)
            kernels[name].update(bound="hbm", achieved_GBs=rate / 1e9, frac=rate / HBM_PEAK)
    if prof:
        dom = max((k for k in prof if k in per), key=lambda k: prof[k][0])
        ms, cnt = prof[dom]
        rate = per[dom] * B * args.steps / (ms * 1e-3)
        roof = {"kernel": dom, "bound": "hbm", "achieved": rate / 1e9, "peak": HBM_PEAK / 1e9, "unit": "GB/s",
                "frac": rate / HBM_PEAK, "traffic": None, "avg_launch_ms": ms / cnt,
                "algorithmic_bytes_per_launch": per[dom] * B * args.steps / cnt}
    result = {
        "metric": f"{alg} wire-field base64 codec, handshakes/sec at batch 2^{lb} per GPU "
                  f"(encode pk_i, pk_r, ct; decode pk_i, ct)",
        "value": value, "unit": "handshakes/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": elapsed * 1e3 / args.steps, "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "u8",
        "data": "synthetic: uniformly random pk / ct bytes of the ML-KEM sizes, device-resident",
        "config": {"workload": f"{alg} KEM wire fields of 2^{lb} exchanges per GPU (SURVEY.md 8f-3)",
                   "alg": alg, "batch_per_gpu": B, "global_batch": B * world, "bytes_per_handshake": bytes_hs,
                   "parallelism": f"index-sharded x{world} (no data-path collective)"},
        "roofline": roof, "hbm_GBs_step": value * bytes_hs / 1e9, "kernels_timed_region": kernels,
        "checks": {"roundtrip_mismatches_or_rejects": bad}, "cpu_baseline": None,
    }
    if rank == 0 and world == 1 and not args.no_cpu:
        import base64
        S = 1 << 14
        h_pk, h_pkr, h_ct = (np.ascontiguousarray(t[:S].cpu().numpy()) for t in (pk_i, pk_r, ct_))
        t0 = time.perf_counter()
        m = 0
        while time.perf_counter() - t0 < 10.0 and m < S:  # the reference call pattern, one field per call
            a = base64.b64encode(h_pk[m].tobytes()).decode()
            base64.b64decode(a)
            c = base64.b64encode(h_ct[m].tobytes()).decode()
            base64.b64encode(h_pkr[m].tobytes()).decode()
            base64.b64decode(c)
            m += 1
        dt = time.perf_counter() - t0
        result["cpu_baseline"] = {"value": m / dt, "unit": "handshakes/s", "cores": 1, "kind": "reference",
                                  "sample": f"{m} handshakes' fields through Python base64 (the reference's own "
                                            f"calls, messaging.py:607, 829, 852-853, 1037), one core"}
    if rank == 0:
        print(json.dumps(result))
    if world > 1:
        dist.destroy_process_group()


def _ctx_profile(obj, on):
    from qrkem._native import LIB
    LIB.qrk_ctx_profile(obj._ctx, int(on))


def _ctx_profile_read(obj):
    import ctypes as ct
    from qrkem._native import LIB
    n = LIB.qrk_ctx_profile_collect(obj._ctx)
    out = {}
    for i in range(max(n, 0)):
        name, ms, cnt = ct.c_char_p(), ct.c_double(), ct.c_uint64()
        LIB.qrk_ctx_profile_get(obj._ctx, i, ct.byref(name), ct.byref(ms), ct.byref(cnt))
        out[name.value.decode()] = (ms.value, cnt.value)
    return out


def launcher_argv(bench_argv, nproc, port, script=None):
    """The child command that runs this bench as `nproc` ranks (one per GPU) when bench.py is
    started without a launcher: torch.distributed.run on 127.0.0.1, same bench arguments."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
            "--master-addr=127.0.0.1", f"--master-port={port}", str(script or ROOT / "bench.py"), *bench_argv]


def launcher_env(environ):
    """Environment of the launched ranks: the caller's, with dmabuf IPC kept (RCCL on this image
    needs HSA_ENABLE_IPC_MODE_LEGACY=0) and no stale rank variables."""
    env = {k: v for k, v in environ.items()
           if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")}
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return env


def pick_json_line(text):
    """The single result line rank 0 printed (the last stdout line that parses as a bench JSON)."""
    found = None
    for line in text.splitlines():
        line = line.strip()
        if line.startswith("{"):
            try:
                d = json.loads(line)
            except ValueError:
                continue
            if isinstance(d, dict) and "metric" in d and "value" in d:
                found = line
    return found


def launch_ranks(nproc, bench_argv, script=None):
    """--gpus N > 1 without WORLD_SIZE: start the N ranks as a child process (this process has
    made no HIP call, and it never execs), relay rank 0's JSON line, exit with the child's code."""
    import socket
    import subprocess
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    proc = subprocess.run(launcher_argv(bench_argv, nproc, port, script), env=launcher_env(os.environ),
                          stdout=subprocess.PIPE, text=True)
    line = pick_json_line(proc.stdout)
    if line is not None:
        print(line)
    elif proc.stdout:
        sys.stdout.write(proc.stdout)
    if proc.returncode == 0 and line is None:
        return 1
    return proc.returncode


def strong_digest_block(world, total):
    """Block of global indices for the strong-scaling shard digests: 2^20 (one library chunk)
    when every shard boundary falls on it, else the largest divisor of 2^20 that every boundary
    shares; None when that is below 2^12 (then one digest per rank is reported instead)."""
    import math

    from qrkem.shard import DIGEST_BLOCK, strong_shard
    g = DIGEST_BLOCK
    for r in range(world):
        g = math.gcd(g, strong_shard(r, world, total).first)
    g = math.gcd(g, total)
    return g if g >= 1 << 12 else None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--alg", default="ML-KEM-768")
    ap.add_argument("--log2-batch", type=int, default=None, help="default 20 (ML-KEM), 16 (FrodoKEM, HQC)")
    ap.add_argument("--chunk", type=int, default=1 << 20)
    ap.add_argument("--global-log2-batch", type=int, default=None,
                    help="BASELINE configs[2]: a fixed global batch of 2^G handshakes split across the ranks "
                         "(strong scaling, e.g. 24), with per-block digests of every rank's (ct, ss)")
    ap.add_argument("--seed", type=lambda x: int(x, 0), default=0x5EED)
    ap.add_argument("--mode", choices=["encdec", "decaps-tampered", "handshake", "wire"], default="encdec")
    ap.add_argument("--symmetric", default="AES-256-GCM", help="handshake mode: HKDF key size / info suffix")
    ap.add_argument("--streams", type=int, default=0, choices=[0, 1],
                    help="library schedule (qrk_ctx_set_streams): 0 multi-role launches, 1 serial "
                         "(one kernel per launch); every kernel runs on the caller's stream in both")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-profile", action="store_true")
    args = ap.parse_args()

    if args.global_log2_batch is not None and (1 << args.global_log2_batch) < args.gpus:
        raise SystemExit(f"--global-log2-batch {args.global_log2_batch}: fewer handshakes than ranks")
    if os.environ.get("WORLD_SIZE") in (None, "") and args.gpus > 1:
        # before any HIP call: no exec, a child (QRK_BENCH_RANK_SCRIPT: a stub rank script, tests only)
        return launch_ranks(args.gpus, sys.argv[1:], script=os.environ.get("QRK_BENCH_RANK_SCRIPT") or None)
    world = env_int("WORLD_SIZE", 1)
    rank = env_int("RANK", 0)
    local = env_int("LOCAL_RANK", 0)
    if world != args.gpus and rank == 0:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE {world}", file=sys.stderr)
    # One rank per GPU over RCCL ("nccl").  QRK_BENCH_BACKEND=gloo with more ranks than GPUs
    # rehearses the multi-rank path on a single card (never used for scaling numbers).
    global RED_DEVICE
    backend = os.environ.get("QRK_BENCH_BACKEND", "nccl")
    ndev = torch.cuda.device_count()
    if backend == "nccl" and local >= ndev:
        raise SystemExit(f"LOCAL_RANK {local} but only {ndev} GPUs visible")
    local %= max(ndev, 1)
    torch.cuda.set_device(local)
    RED_DEVICE = f"cuda:{local}" if backend == "nccl" else None
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)

    if args.mode == "handshake":
        return bench_handshake(args, world, rank, local)
    if args.mode == "wire":
        return bench_wire(args, world, rank, local)
    from qrkem.batch import BatchKEM
    from qrkem.shard import block_digests, combine_digests, gather_digests, reduce_run, strong_shard, weak_shard
    alg = args.alg
    frodo = alg in FP
    hqc = alg in HQ
    lb = args.log2_batch if args.log2_batch is not None else (16 if (frodo or hqc) else 20)
    B = 1 << lb
    strong = args.global_log2_batch is not None
    if strong:  # configs[2]: 2^G handshakes in total, contiguous index shards
        if args.mode != "encdec":
            raise SystemExit("--global-log2-batch: encdec mode only")
        lb = args.global_log2_batch
        shard = strong_shard(rank, world, 1 << lb)
    else:  # weak scaling: 2^lb handshakes per rank, rank r takes [r 2^lb, (r+1) 2^lb)
        shard = weak_shard(rank, world, B)
    B = shard.count
    eng = BatchKEM(alg, device=local, chunk=args.chunk)
    eng.set_streams(args.streams)
    cap = eng.effective_chunk
    nch = -(-B // cap)
    chunk_eff = min(cap, (-(-B // nch) + 63) // 64 * 64)  # equal chunks, as the library splits them
    base = shard.first  # global index range [base, base + B)

    kpl, encl = eng.kp_coins, eng.enc_coins
    if kpl + encl <= 136:  # one SHAKE256 block per index
        coins = eng.bench_coins(B, kpl + encl, args.seed, base)
        kc = coins[:, :kpl].contiguous()
        ec = coins[:, kpl:].contiguous()
        del coins
    else:  # HQC-192/256: KeyGen and Encaps coins from two seeds
        kc = eng.bench_coins(B, kpl, args.seed, base)
        ec = eng.bench_coins(B, encl, args.seed ^ 0xE7C, base)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    pk, sk = eng.keypair(coins=kc)
    torch.cuda.synchronize()
    keygen_s = time.perf_counter() - t0

    def barrier():
        if world > 1:
            dist.barrier()

    def timed(step, profile=False):
        for _ in range(args.warmup):
            step()
        torch.cuda.synchronize()
        if profile:  # live HIP-event kernel timing over the timed steps only
            eng.profile(True)
        barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            out = step()
        torch.cuda.synchronize()
        barrier()
        return time.perf_counter() - t0, out

    checks = {}
    variants = {}
    if args.mode == "encdec":
        def step():
            ct_, ss_ = eng.encaps(pk, coins=ec)
            return ct_, ss_, eng.decaps(sk, ct_)
        main_step = step
    else:
        ct_valid, ss0 = eng.encaps(pk, coins=ec)
        cts = {"all-valid": ct_valid}
        for name, m in (("all-tampered", 1), ("mixed", 2)):
            c = ct_valid.clone()
            eng.tamper(c, args.seed, m)
            cts[name] = c
        torch.cuda.synchronize()
        for name in ("all-valid", "all-tampered"):
            el, _ = timed(lambda c=cts[name]: eng.decaps(sk, c))
            variants[name] = el * 1e3 / args.steps

        def main_step():
            return cts["mixed"], ss0, eng.decaps(sk, cts["mixed"])

    elapsed, out = timed(main_step, profile=not args.no_profile)
    prof_live = eng.profile_read() if not args.no_profile else {}
    eng.profile(False)
    # Kernel-in-isolation pass (serial schedule, one untimed step: qrk_ctx_set_streams(1) runs
    # one kernel per launch, the SampleNTT fix-up included), since the multi-role launches of the
    # timed region time two kernels as one.
    prof = {}
    if not args.no_profile:
        eng.set_streams(1)
        eng.profile(True)
        main_step()
        torch.cuda.synchronize()
        prof = dict(eng.profile_read().items())
        eng.profile(False)
        eng.set_streams(args.streams)

    ct, ss, ss2 = out
    if args.mode == "encdec":
        bad = int((ss != ss2).any(dim=1).sum().item())
        counters = [bad, 0]
    else:
        variants["mixed"] = elapsed * 1e3 / args.steps
        tampered = (ct != cts["all-valid"]).any(dim=1)
        same = (ss2 == ss).all(dim=1)
        if hqc:  # the per-record return code must flag exactly the tampered rows
            _, st = eng.decaps(sk, cts["mixed"], return_status=True)
            checks["status_mismatches"] = int(((st != 0) != tampered).sum().item())
        # valid rows must give the encapsulated key, tampered rows the implicit-rejection key
        bad = int((same != ~tampered).sum().item())
        counters = [bad, int(tampered.sum().item())]
    elapsed, (bad, n_tampered) = reduce_run(elapsed, counters, device=RED_DEVICE)
    if args.mode == "encdec":
        checks["ss_enc_eq_ss_dec_mismatches"] = bad
    else:
        checks["implicit_rejection_mismatches"] = bad
        checks["tampered"] = n_tampered
        checks["decaps_ms_per_step"] = variants
        checks["tampered_over_valid_time"] = variants["all-tampered"] / variants["all-valid"]

    total = (1 << lb if strong else B * world) * args.steps
    value = total / elapsed
    ms_per_step = elapsed * 1e3 / args.steps
    # roofline: kernel durations measured live over the timed region (the schedule as run);
    # "kernels" additionally reports the serial-schedule pass (kernels in isolation)
    _, roof, mfma = kernel_report(alg, args.mode, prof_live, B * args.steps)
    kernels, roof_iso, _ = kernel_report(alg, args.mode, prof, B)
    if roof is not None:
        if mfma is not None:
            mfma["counters"] = pmc_mfma(alg, args.mode, chunk_eff, mfma["kernel"].split()[0])
        tb, src = pmc_traffic(alg, args.mode, chunk_eff, roof["kernel"])
        roof["traffic"] = tb
        roof["traffic_unit"] = ("HBM bytes per launch: rocprofv3 FETCH_SIZE x 2 + WRITE_SIZE; the x 2 is calibrated on "
                                "this library's own read patterns (0.500 for every coalesced width, 4-16 B/lane and the "
                                "cores' 64-B runs; 0.774 for lane-per-record AoS reads, i.e. real over-fetch) and "
                                "WRITE_SIZE reads exact (profiles/r3/fetch_calibration.json)")
        roof["traffic_source"] = src
        roof["algorithmic_ops_per_launch"] = roof.pop("ops_per_launch")
        roof["isolated_frac"] = roof_iso["frac"] if roof_iso and roof_iso["kernel"] == roof["kernel"] else None
        iss, iss_src = pmc_issued(alg, args.mode, chunk_eff, roof["kernel"])
        if roof["bound"] == "valu" and iss:
            # every issued VALU instruction x 64 lanes over the isolated kernel time (rocprofv3 PMC)
            roof["issued"] = {"Tops": iss, "frac": iss * 1e12 / VALU_PEAK, "full_rate_ceiling_Tops": VALU_FULL_RATE,
                              "frac_of_full_rate_ceiling": iss / VALU_FULL_RATE, "source": iss_src}
        kp = keccak_practical_peak()
        if roof["bound"] == "valu" and kp:
            # the measured ceiling of the Keccak instruction mix (half-rate v_alignbit), see DESIGN.md 7
            roof["practical_peak"] = kp
            roof["practical_frac"] = roof["achieved"] / kp
            if roof["isolated_frac"] is not None:
                roof["practical_isolated_frac"] = roof["isolated_frac"] * roof["peak"] / kp

    W = valu_ops(alg, args.mode)
    headline = alg == "ML-KEM-768" and args.mode == "encdec"
    cfg_idx = (2 if strong else 1) if not frodo and args.mode == "encdec" else (3 if frodo else 4)
    cfg_label = "SURVEY.md 8f-4" if hqc else f"BASELINE.json configs[{cfg_idx}]"
    what = "Encaps+Decaps" if args.mode == "encdec" else "Decaps, 50% tampered (mixed)"
    result = {
        "metric": (f"{alg} encaps+decaps/sec (node) at a fixed global batch of 2^{lb} sharded across the GPUs"
                   if strong else METRIC if headline else
                   f"{alg} {'encaps+decaps' if args.mode == 'encdec' else 'decaps'}/sec at batch 2^{lb} per GPU"),
        "value": value,
        "unit": "encaps+decaps/s" if args.mode == "encdec" else "decaps/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_per_step,
        "higher_is_better": True,
        "scaling": "strong" if strong else "weak",
        "vs_baseline": None,
        "dtype": "u32 (Keccak, F2[X] words, GF(2^8))" if hqc else "u32" if not frodo else ("u32 (AES T-table) + i8->i32 (MFMA)" if alg.endswith("-AES") else "u32 (Keccak) + i8->i32 (MFMA)"),
        "data": "synthetic: coins = SHAKE256('qrk-bench'||LE64(seed)||LE64(i)) generated on device; "
                "keys from batched KeyGen on those coins",
        "config": {"workload": (f"{alg} {what} of 2^{lb} device-resident handshakes in total, "
                                f"2^{lb}/{world} per GPU ({cfg_label})" if strong else
                                f"{alg} {what} of 2^{lb} device-resident handshakes per GPU ({cfg_label})"),
                   "alg": alg, "batch_per_gpu": B, "global_batch": (1 << lb) if strong else B * world,
                   "first_index": base, "chunk": chunk_eff,
                   "parallelism": f"index-sharded x{world} (no data-path collective)"},
        "roofline": roof,
        "mfma": mfma,
        "valu_frac_of_peak_step": value * W / (VALU_PEAK * world),  # per GPU
        "valu_ops_per_unit": W,
        "keygen_per_s": B * world / keygen_s if keygen_s > 0 else None,
        "kernels": kernels,
        "kernels_timed_region": {k: {"avg_ms": ms / c, "launches": c} for k, (ms, c) in prof_live.items()},
        "checks": checks,
        "cpu_baseline": None,
    }
    if strong:
        # per-record SHA3-256(ct_i || ss_i) on the GPU, SHA-256 per block of 2^20 global indices:
        # the same block digests for every GPU count
        recs = eng.digest_rows(ct, ss).cpu().numpy()
        dblock = strong_digest_block(world, 1 << lb)
        if dblock is not None:
            mine = block_digests(recs, base, dblock)
        else:  # shards not aligned to any block of >= 2^12 indices: one digest per rank
            import hashlib
            mine = {rank: hashlib.sha256(np.ascontiguousarray(recs).tobytes()).hexdigest()}
        allb = gather_digests(mine)
        result["shard_digests"] = {
            "record": "SHA3-256(ct_i || ss_i)", "block": dblock if dblock is not None else "per-rank",
            "block_digest": ("SHA-256 over the block's record digests in index order" if dblock is not None else
                             "SHA-256 over each rank's record digests (depends on the GPU count)"),
            "blocks": {str(k): v for k, v in sorted(allb.items())},
            "global": combine_digests(allb), "rank0_blocks": sorted(mine)}
    if rank == 0 and world == 1 and not args.no_cpu:
        result["cpu_baseline"] = cpu_baseline(alg, args.mode, kc, pk, sk, ec, ct, ss2 if args.mode != "encdec" else ss,
                                              B)
    if rank == 0:
        print(json.dumps(result))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    sys.exit(main())
