"""Batched wire-format codec for KEM payloads.

The reference carries every KEM payload as standard base64 text inside JSON
(``quantum_resistant_p2p/app/messaging.py:607`` initiator public key,
``:852-853`` ciphertext and responder public key) and decodes it with
``base64.b64decode`` (``:829``).  :class:`Base64Codec` runs that for N records per
call on the GPU (``wire.hip``); JSON assembly, signatures and TCP framing stay on the
host (out of scope).
"""
from __future__ import annotations

import ctypes as ct

from ._native import LIB, last_error
from .batch import _is_dev

try:
    import torch
except ImportError:  # pragma: no cover
    torch = None


def encoded_len(n_bytes: int) -> int:
    """Characters of the padded base64 text of n_bytes bytes."""
    return 4 * ((n_bytes + 2) // 3)


class Base64Codec:
    def __init__(self, device: int = 0):
        self.device = device
        h = ct.c_void_p()
        if LIB.qrk_ctx_create(ct.byref(h), device) != 0:
            raise RuntimeError(f"qrkem: cannot create a context on device {device}: {last_error()}")
        self._ctx = h

    def close(self) -> None:
        if getattr(self, "_ctx", None):
            LIB.qrk_ctx_destroy(self._ctx)
            self._ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _stream(self, t):
        return ct.c_void_p(torch.cuda.current_stream(t.device).cuda_stream)

    def encode(self, data):
        """data: cuda uint8 [n, L] -> cuda uint8 [n, 4 ceil(L/3)] (ASCII, no separators)."""
        if not _is_dev(data) or data.dtype != torch.uint8 or data.dim() != 2:
            raise ValueError("expected a cuda uint8 [n, L] tensor")
        data = data.contiguous()
        n, L = data.shape
        out = torch.empty((n, encoded_len(L)), dtype=torch.uint8, device=data.device)
        rc = LIB.qrk_base64_encode_batch(self._ctx, n, ct.c_void_p(data.data_ptr()), L,
                                         ct.c_void_p(out.data_ptr()), self._stream(data))
        if rc != 0:
            raise RuntimeError(f"qrkem base64 encode failed: {last_error()}")
        return out

    def decode(self, text, out_len: int):
        """text: cuda uint8 [n, 4 ceil(out_len/3)] -> (cuda uint8 [n, out_len], int32 [n] status:
        0 ok, -1 malformed record)."""
        if not _is_dev(text) or text.dtype != torch.uint8 or text.dim() != 2:
            raise ValueError("expected a cuda uint8 [n, chars] tensor")
        if text.shape[1] != encoded_len(out_len):
            raise ValueError(f"{out_len}-byte records take {encoded_len(out_len)} characters, got {text.shape[1]}")
        text = text.contiguous()
        n = text.shape[0]
        out = torch.empty((n, out_len), dtype=torch.uint8, device=text.device)
        status = torch.empty((n,), dtype=torch.int32, device=text.device)
        rc = LIB.qrk_base64_decode_batch(self._ctx, n, ct.c_void_p(text.data_ptr()), out_len,
                                         ct.c_void_p(out.data_ptr()), ct.c_void_p(status.data_ptr()),
                                         self._stream(text))
        if rc != 0:
            raise RuntimeError(f"qrkem base64 decode failed: {last_error()}")
        return out, status


def to_strings(text) -> list:
    """[n, chars] uint8 (device or host) -> list of str, the JSON field values."""
    a = text.cpu().numpy() if _is_dev(text) else text
    return [row.tobytes().decode("ascii") for row in a]
