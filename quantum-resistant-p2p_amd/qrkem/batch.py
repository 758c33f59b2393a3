"""Batched KEM engine: N independent handshakes per call on one MI355X.

The reference performs one ``OQS_KEM_*`` call per handshake on the asyncio
thread (``quantum_resistant_p2p/crypto/key_exchange.py:133,155-156,178-179``).
:class:`BatchKEM` runs N of them per call through ``qrk_kem_*_batch`` in
libqrkem.so.  Device tensors (``torch.uint8`` on ``cuda``) are passed by pointer
and processed on the caller's current stream (zero copy); host arrays go through
the synchronous ``*_batch_host`` entry points.

Tensors are contiguous ``[n, len]`` uint8 -- the AoS layout the C ABI documents.
"""
from __future__ import annotations

import ctypes as ct
from typing import Optional

import numpy as np

from ._native import LIB, last_error
from .oqs import MechanismNotEnabledError, MechanismNotSupportedError, get_enabled_kem_mechanisms, \
    get_supported_kem_mechanisms, kem_sizes

try:  # torch is plumbing for device memory/streams, not a compute path
    import torch
except ImportError:  # pragma: no cover
    torch = None


def _is_dev(x) -> bool:
    return torch is not None and isinstance(x, torch.Tensor) and x.is_cuda


def _dptr(t) -> ct.c_void_p:
    assert t.dtype == torch.uint8 or t.dtype == torch.int32, t.dtype
    assert t.is_contiguous()
    return ct.c_void_p(t.data_ptr())


def _check_dev(t, width: int, what: str, n: Optional[int] = None):
    """Device [n, width] uint8 contiguous, like _as_host's check for host arrays: the kernels
    index rows at the fixed stride `width`, so a wrong shape must fail here, not read past
    the tensor (the reference raises ValueError on a wrong-length input, oqs.py:341-347)."""
    if t.dtype != torch.uint8 or t.dim() != 2 or t.shape[1] != width:
        raise ValueError(f"{what}: expected a [n, {width}] uint8 tensor, got {tuple(t.shape)} {t.dtype}")
    if n is not None and t.shape[0] != n:
        raise ValueError(f"{what}: batch size {t.shape[0]} != {n}")
    if not t.is_contiguous():
        raise ValueError(f"{what}: tensor must be contiguous")
    return t


def _hptr(a: np.ndarray) -> ct.c_void_p:
    assert a.flags["C_CONTIGUOUS"]
    return a.ctypes.data_as(ct.c_void_p)


def _as_host(x, width: int) -> np.ndarray:
    if isinstance(x, (bytes, bytearray)):
        x = np.frombuffer(bytes(x), np.uint8).reshape(1, -1)
    elif isinstance(x, (list, tuple)):
        x = np.stack([np.frombuffer(bytes(b), np.uint8) for b in x]) if x else np.zeros((0, width), np.uint8)
    a = np.ascontiguousarray(np.asarray(x, dtype=np.uint8))
    if a.ndim != 2 or a.shape[1] != width:
        raise ValueError(f"expected a [n, {width}] uint8 array, got shape {a.shape}")
    return a


class BatchKEM:
    """Batched KeyGen / Encaps / Decaps for one algorithm on one device."""

    def __init__(self, alg: str, device: int = 0, chunk: Optional[int] = None):
        if alg not in get_enabled_kem_mechanisms():
            if alg in get_supported_kem_mechanisms():
                raise MechanismNotEnabledError(alg)
            raise MechanismNotSupportedError(alg)
        self.alg = alg
        self._name = alg.encode()
        self.device = device
        s = kem_sizes(alg)
        self.pk_len = s["length_public_key"]
        self.sk_len = s["length_secret_key"]
        self.ct_len = s["length_ciphertext"]
        self.ss_len = s["length_shared_secret"]
        self.kp_coins = s["length_keypair_coins"]
        self.enc_coins = s["length_encaps_coins"]
        h = ct.c_void_p()
        if LIB.qrk_ctx_create(ct.byref(h), device) != 0:
            raise RuntimeError(f"qrkem: cannot create a context on device {device}: {last_error()}")
        self._ctx = h
        if chunk:
            LIB.qrk_ctx_set_chunk(self._ctx, chunk)

    def close(self) -> None:
        if getattr(self, "_ctx", None):
            LIB.qrk_ctx_destroy(self._ctx)
            self._ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _stream(self):
        return ct.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)

    def _check(self, rc: int, what: str) -> None:
        if rc != 0:
            raise RuntimeError(f"qrkem {what} failed ({self.alg}): {last_error()}")

    def _empty(self, n: int, width: int):
        return torch.empty((n, width), dtype=torch.uint8, device=f"cuda:{self.device}")

    # ------------------------------------------------------------------ KeyGen
    def keypair(self, n: Optional[int] = None, coins=None):
        """Returns (pk [n, pk_len], sk [n, sk_len]).  ``coins`` [n, kp_coins] or None (OS CSPRNG).

        Device coins (or ``n`` without coins) -> device outputs; host coins -> numpy outputs."""
        if coins is None and n is None:
            raise ValueError("give n or coins")
        if coins is not None and not _is_dev(coins):
            c = _as_host(coins, self.kp_coins)
            n = c.shape[0]
            pk = np.zeros((n, self.pk_len), np.uint8)
            sk = np.zeros((n, self.sk_len), np.uint8)
            self._check(LIB.qrk_kem_keypair_batch_host(self._ctx, self._name, n, _hptr(pk), _hptr(sk), _hptr(c)),
                        "keypair")
            return pk, sk
        if coins is not None:
            n = _check_dev(coins, self.kp_coins, "keypair coins").shape[0]
        pk, sk = self._empty(n, self.pk_len), self._empty(n, self.sk_len)
        cp = _dptr(coins) if coins is not None else None
        self._check(LIB.qrk_kem_keypair_batch(self._ctx, self._name, n, _dptr(pk), _dptr(sk), cp, self._stream()),
                    "keypair")
        return pk, sk

    # ------------------------------------------------------------------ Encaps
    def encaps(self, pk, coins=None, return_status: bool = False):
        """Returns (ct, ss) (+ status int32[n]: -1 where pk fails the FIPS 203 7.2 check)."""
        if _is_dev(pk):
            n = _check_dev(pk, self.pk_len, "encaps pk").shape[0]
            c, ss = self._empty(n, self.ct_len), self._empty(n, self.ss_len)
            st = torch.empty((n,), dtype=torch.int32, device=pk.device) if return_status else None
            if coins is not None and not _is_dev(coins):
                coins = torch.from_numpy(_as_host(coins, self.enc_coins)).to(pk.device)
            if coins is not None:
                _check_dev(coins, self.enc_coins, "encaps coins", n)
            self._check(LIB.qrk_kem_encaps_batch(self._ctx, self._name, n, _dptr(c), _dptr(ss), _dptr(pk),
                                                 _dptr(coins) if coins is not None else None,
                                                 _dptr(st) if st is not None else None, self._stream()), "encaps")
            return (c, ss, st) if return_status else (c, ss)
        p = _as_host(pk, self.pk_len)
        n = p.shape[0]
        c = np.zeros((n, self.ct_len), np.uint8)
        ss = np.zeros((n, self.ss_len), np.uint8)
        st = np.zeros((n,), np.int32)
        cc = _as_host(coins, self.enc_coins) if coins is not None else None
        self._check(LIB.qrk_kem_encaps_batch_host(self._ctx, self._name, n, _hptr(c), _hptr(ss), _hptr(p),
                                                  _hptr(cc) if cc is not None else None, _hptr(st)), "encaps")
        return (c, ss, st) if return_status else (c, ss)

    # ------------------------------------------------------------------ Decaps
    def decaps(self, sk, ct_, return_status: bool = False):
        """Returns ss [n, ss_len] (+ status int32[n] with return_status).  ML-KEM / FrodoKEM:
        implicit rejection, status 0.  HQC: status -1 where the re-encryption check fails (the
        OQS_ERROR liboqs returns there); ss = K(sigma || ct) is written either way."""
        if _is_dev(sk) and _is_dev(ct_):
            n = _check_dev(sk, self.sk_len, "decaps sk").shape[0]
            _check_dev(ct_, self.ct_len, "decaps ct", n)
            ss = self._empty(n, self.ss_len)
            if return_status:
                st = torch.empty((n,), dtype=torch.int32, device=sk.device)
                self._check(LIB.qrk_kem_decaps_batch_status(self._ctx, self._name, n, _dptr(ss), _dptr(ct_),
                                                            _dptr(sk), _dptr(st), self._stream()), "decaps")
                return ss, st
            self._check(LIB.qrk_kem_decaps_batch(self._ctx, self._name, n, _dptr(ss), _dptr(ct_), _dptr(sk),
                                                 self._stream()), "decaps")
            return ss
        s = _as_host(sk, self.sk_len)
        c = _as_host(ct_, self.ct_len)
        if s.shape[0] != c.shape[0]:
            raise ValueError("sk and ct batch sizes differ")
        ss = np.zeros((s.shape[0], self.ss_len), np.uint8)
        st = np.zeros((s.shape[0],), np.int32)
        self._check(LIB.qrk_kem_decaps_batch_status_host(self._ctx, self._name, s.shape[0], _hptr(ss), _hptr(c),
                                                         _hptr(s), _hptr(st)), "decaps")
        return (ss, st) if return_status else ss

    @property
    def effective_chunk(self) -> int:
        """Handshakes per internal chunk for this algorithm (FrodoKEM caps it by scratch size)."""
        return int(LIB.qrk_ctx_effective_chunk(self._ctx, self.alg.encode()))

    @property
    def scratch_bytes(self) -> int:
        """Device scratch the context holds (grown on demand, never shrunk)."""
        return int(LIB.qrk_ctx_scratch_bytes(self._ctx))

    def set_streams(self, streams: int) -> None:
        """0 (default): independent kernels of one operation share multi-role launches; 1: serial,
        one kernel per launch (per-kernel timings in isolation).  Every kernel runs on the caller's
        stream in both schedules."""
        self._check(LIB.qrk_ctx_set_streams(self._ctx, streams), "set_streams")

    # ------------------------------------------------------------------ kernel timing
    def profile(self, enable: bool = True) -> None:
        """Reset and enable/disable per-kernel HIP-event timing on the launch stream."""
        self._check(LIB.qrk_ctx_profile(self._ctx, int(enable)), "profile")

    def profile_read(self) -> dict:
        """{kernel name: (total ms, launches)} accumulated since profile(True)."""
        n = LIB.qrk_ctx_profile_collect(self._ctx)
        if n < 0:
            raise RuntimeError(f"qrkem profile collect failed: {last_error()}")
        out = {}
        for i in range(n):
            name, ms, cnt = ct.c_char_p(), ct.c_double(), ct.c_uint64()
            self._check(LIB.qrk_ctx_profile_get(self._ctx, i, ct.byref(name), ct.byref(ms), ct.byref(cnt)),
                        "profile_get")
            out[name.value.decode()] = (ms.value, cnt.value)
        return out

    # ------------------------------------------------------------------ bench helpers
    def bench_coins(self, n: int, length: int, seed: int, first: int = 0):
        out = self._empty(n, length)
        self._check(LIB.qrk_bench_coins(self._ctx, n, length, seed, first, _dptr(out), self._stream()),
                    "bench_coins")
        return out

    def digest_rows(self, a, b=None):
        """Per-record SHA3-256(a_i || b_i) of device tensors [n, la] / [n, lb] -> [n, 32] uint8
        (qrk_digest_rows): the records the sharded bench combines into shard digests."""
        n = a.shape[0]
        _check_dev(a, a.shape[1], "digest a")
        if b is not None:
            _check_dev(b, b.shape[1], "digest b", n)
        out = self._empty(n, 32)
        self._check(LIB.qrk_digest_rows(self._ctx, n, _dptr(a), a.shape[1], _dptr(b) if b is not None else None,
                                        b.shape[1] if b is not None else 0, _dptr(out), self._stream()),
                    "digest_rows")
        return out

    def cleanse(self) -> None:
        """Zero every context buffer that can hold keys or secret intermediates (qrk_ctx_cleanse)."""
        self._check(LIB.qrk_ctx_cleanse(self._ctx), "cleanse")

    def tamper(self, ct_, seed: int, mode: int) -> None:
        """In-place: mode 0 none, 1 every ciphertext, 2 Bernoulli(1/2) per index."""
        _check_dev(ct_, self.ct_len, "tamper ct")
        self._check(LIB.qrk_tamper(self._ctx, ct_.shape[0], self.ct_len, seed, mode, _dptr(ct_), self._stream()),
                    "tamper")

    def hqc_supports(self, r, kind: int):
        """HQC fixed-weight supports from device uint32 random words r [n][weight] (kind 0: w,
        1: w_r = w_e), duplicates removed as the spec does (test hook, qrk_hqc_supports)."""
        out = torch.empty_like(r)
        self._check(LIB.qrk_hqc_supports(self._ctx, self.alg.encode(), kind, r.shape[0], _dptr(r), _dptr(out),
                                          self._stream()), "hqc_supports")
        return out
