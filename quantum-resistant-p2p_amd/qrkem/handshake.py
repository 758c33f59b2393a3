"""Batched protocol handshakes and key derivation.

The reference completes one key exchange per peer on the asyncio thread
(``quantum_resistant_p2p/app/messaging.py``):

* initiator ``initiate_key_exchange`` -- ephemeral KeyGen (``:590``);
* responder ``_handle_key_exchange_init`` -- its own ephemeral KeyGen (``:809``, the
  public key is sent back at ``:853`` but never used for the KEM), Encaps of the
  initiator's key (``:830``), ``_derive_symmetric_key`` (``:845``);
* initiator ``_handle_key_exchange_response`` -- Decaps (``:1038``),
  ``_derive_symmetric_key`` (``:1068``).

``_derive_symmetric_key`` (``:350-382``) is HKDF-SHA256 with ``salt=None``,
``length=symmetric.key_size`` and ``info = b"quantum_resistant_p2p-v1-{a}-{b}-{sym}"``
over the alphabetically sorted node ids.

:class:`KeyDerivation` is the batched drop-in for ``_derive_symmetric_key``;
:class:`HandshakeDriver` runs N complete exchanges with exactly that operation mix in
one call (``qrk_handshake_batch``).  Both run on the GPU only (hkdf.hip, mlkem.hip,
frodo.hip); there is no CPU path.
"""
from __future__ import annotations

import ctypes as ct
from dataclasses import dataclass
from typing import Optional, Sequence, Union

import numpy as np

from ._native import LIB, last_error
from .batch import BatchKEM, _as_host, _is_dev

try:
    import torch
except ImportError:  # pragma: no cover
    torch = None

# crypto/symmetric.py:70-81 (AES-256-GCM) and :168-179 (ChaCha20-Poly1305): 32-byte keys
SYMMETRIC_KEY_SIZE = {"AES-256-GCM": 32, "ChaCha20-Poly1305": 32}


def protocol_info(node_id: str, peer_id: str, symmetric_name: str) -> bytes:
    """The HKDF info of messaging.py:364-367 (ids sorted so both peers agree)."""
    a, b = sorted([node_id, peer_id])
    return f"quantum_resistant_p2p-v1-{a}-{b}-{symmetric_name}".encode()


def pack_infos(infos: Sequence[bytes]) -> tuple[np.ndarray, np.ndarray]:
    """list of byte strings -> (concatenated uint8 bytes, uint64 offsets [n+1])."""
    off = np.zeros(len(infos) + 1, np.uint64)
    if len(infos):
        off[1:] = np.cumsum([len(x) for x in infos], dtype=np.uint64)
    data = np.frombuffer(b"".join(infos) or b"\0", np.uint8).copy()
    return data, off


def _ptr(t) -> ct.c_void_p:
    if t is None:
        return None
    if _is_dev(t):
        assert t.is_contiguous()
        return ct.c_void_p(t.data_ptr())
    assert t.flags["C_CONTIGUOUS"]
    return t.ctypes.data_as(ct.c_void_p)


def _dev(a: np.ndarray, device: int):
    return torch.from_numpy(np.array(a, copy=True, order="C")).to(f"cuda:{device}")


class PackedInfos:
    """Per-key HKDF info resident on the device: one shared byte string, or one per key
    (concatenated bytes + uint64 offsets).  Build once and reuse across calls."""

    def __init__(self, infos: Union[bytes, Sequence[bytes]], n: int, device: int):
        self.n = n
        if isinstance(infos, (bytes, bytearray)):
            self.data = _dev(np.frombuffer(bytes(infos) or b"\0", np.uint8), device)
            self.off = None
            self.length = len(infos)
        else:
            if len(infos) != n:
                raise ValueError(f"{len(infos)} info strings for {n} keys")
            data, off = pack_infos([bytes(x) for x in infos])
            self.data = _dev(data, device)
            self.off = _dev(off.view(np.int64), device)
            self.length = 0


class KeyDerivation:
    """Batched ``SecureMessaging._derive_symmetric_key`` (messaging.py:350-382)."""

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

    def derive(self, shared_secrets, infos: Union[bytes, Sequence[bytes]], length: int = 32,
               salt: Optional[bytes] = None):
        """okm[i] = HKDF-SHA256(salt, shared_secrets[i], infos[i], length).

        ``shared_secrets``: [n, ss_len] uint8 (torch on cuda -> result on cuda; numpy or a
        list of bytes -> numpy).  ``infos``: one byte string for every key, or one per key."""
        host = not _is_dev(shared_secrets)
        if host:
            if isinstance(shared_secrets, (bytes, bytearray)):
                shared_secrets = [shared_secrets]
            width = len(shared_secrets[0]) if len(shared_secrets) else 32
            ikm = _dev(_as_host(shared_secrets, width), self.device)
        else:
            ikm = shared_secrets.contiguous()
        n, ikm_len = ikm.shape
        inf = infos if isinstance(infos, PackedInfos) else PackedInfos(infos, n, self.device)
        okm = torch.empty((n, length), dtype=torch.uint8, device=ikm.device)
        salt_t = _dev(np.frombuffer(salt, np.uint8), self.device) if salt else None
        stream = ct.c_void_p(torch.cuda.current_stream(ikm.device).cuda_stream)
        rc = LIB.qrk_hkdf_sha256_batch(self._ctx, n, _ptr(ikm), ikm_len, _ptr(salt_t), len(salt) if salt else 0,
                                       _ptr(inf.data), _ptr(inf.off), inf.length, _ptr(okm), length, stream)
        if rc != 0:
            raise RuntimeError(f"qrkem HKDF-SHA256 failed: {last_error()}")
        if host:
            return okm.cpu().numpy()
        return okm


@dataclass
class HandshakeBatch:
    """Wire messages and derived keys of N exchanges (device tensors)."""
    pk_initiator: "torch.Tensor"   # key_exchange_init payload (messaging.py:606-616)
    pk_responder: "torch.Tensor"   # responder_public_key (messaging.py:853)
    ciphertext: "torch.Tensor"     # key_exchange_response payload (messaging.py:850-861)
    key_initiator: "torch.Tensor"  # shared_keys[peer] on the initiator (messaging.py:1068)
    key_responder: "torch.Tensor"  # shared_keys[peer] on the responder (messaging.py:845)
    agree: "torch.Tensor"          # int32 [n]: 1 where both sides hold the same key


class HandshakeDriver:
    """N complete key exchanges per call with the reference's operation mix.

    ``kem``: a liboqs algorithm name ("ML-KEM-768") or a key-exchange plugin
    (``MLKEMKeyExchange`` / ``FrodoKEMKeyExchange``; its ``variant`` is used)."""

    def __init__(self, kem, symmetric_name: str = "AES-256-GCM", device: int = 0, chunk: Optional[int] = None):
        alg = kem if isinstance(kem, str) else kem.variant
        if symmetric_name not in SYMMETRIC_KEY_SIZE:
            raise ValueError(f"unknown symmetric algorithm {symmetric_name!r}")
        self.symmetric_name = symmetric_name
        self.key_len = SYMMETRIC_KEY_SIZE[symmetric_name]
        self.engine = BatchKEM(alg, device=device, chunk=chunk)
        self.alg = alg
        self.device = device

    def info_for(self, node_id: str, peer_id: str) -> bytes:
        return protocol_info(node_id, peer_id, self.symmetric_name)

    def pack(self, infos: Union[bytes, Sequence[bytes]], n: Optional[int] = None) -> PackedInfos:
        """Upload HKDF infos once (for repeated :meth:`run` calls over the same peers)."""
        return PackedInfos(infos, n if n is not None else len(infos), self.device)

    def run(self, infos: Union[bytes, Sequence[bytes]], n: Optional[int] = None, coins_kp_initiator=None,
            coins_kp_responder=None, coins_encaps=None) -> HandshakeBatch:
        """Run the exchanges.  ``infos``: one HKDF info for all, one per handshake
        (see :meth:`info_for`), or a :class:`PackedInfos`.  Coins (device uint8 [n, len] or None = OS CSPRNG)."""
        e = self.engine
        if n is None:
            if isinstance(infos, (bytes, bytearray)):
                raise ValueError("give n with a shared info string")
            n = infos.n if isinstance(infos, PackedInfos) else len(infos)
        coins = []
        for c, width in ((coins_kp_initiator, e.kp_coins), (coins_kp_responder, e.kp_coins),
                         (coins_encaps, e.enc_coins)):
            if c is not None and not _is_dev(c):
                c = _dev(_as_host(c, width), self.device)
            if c is not None and tuple(c.shape) != (n, width):
                raise ValueError(f"coins must be [{n}, {width}]")
            coins.append(c)
        inf = infos if isinstance(infos, PackedInfos) else PackedInfos(infos, n, self.device)
        if inf.off is not None and inf.n != n:
            raise ValueError(f"{inf.n} info strings for {n} handshakes")
        out = HandshakeBatch(e._empty(n, e.pk_len), e._empty(n, e.pk_len), e._empty(n, e.ct_len),
                             e._empty(n, self.key_len), e._empty(n, self.key_len),
                             torch.empty((n,), dtype=torch.int32, device=f"cuda:{self.device}"))
        rc = LIB.qrk_handshake_batch(e._ctx, e._name, n, *[_ptr(c) for c in coins], _ptr(inf.data), _ptr(inf.off),
                                     inf.length, self.key_len, _ptr(out.pk_initiator), _ptr(out.pk_responder),
                                     _ptr(out.ciphertext), _ptr(out.key_initiator), _ptr(out.key_responder),
                                     _ptr(out.agree), e._stream())
        if rc != 0:
            raise RuntimeError(f"qrkem handshake batch failed ({self.alg}): {last_error()}")
        return out
