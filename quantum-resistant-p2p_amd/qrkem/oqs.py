"""liboqs-style KEM wrapper over libqrkem.so.

Same public surface as the reference's vendored wrapper for the KEM half
(``quantum_resistant_p2p/vendor/oqs.py:209-421``): ``KeyEncapsulation`` with
``generate_keypair`` / ``export_secret_key`` / ``encap_secret`` /
``decap_secret`` / ``free``, the two mechanism exceptions, and the
``get_enabled_kem_mechanisms`` / ``get_supported_kem_mechanisms`` registry --
so ``quantum_resistant_p2p/crypto/key_exchange.py`` runs on top of it unchanged.

Differences, all deliberate:
* the struct is not a ctypes.Structure subclass; lengths are read through the
  C ABI (``qrk_kem_sizes``) instead of dereferencing ``OQS_KEM*``;
* each call is one handshake on the GPU (batch of one); the batched engine is
  :mod:`qrkem.batch`;
* ``encap_secret(public_key)`` reproduces ctypes ``create_string_buffer``
  semantics of the reference (``oqs.py:338-341``): a shorter key is
  zero-padded, a longer one raises ``ValueError``.
"""
from __future__ import annotations

import ctypes as ct
from typing import Union

from ._native import LIB, last_error

OQS_SUCCESS = 0
OQS_ERROR = -1


def oqs_version() -> str:
    return LIB.OQS_version().decode()


class MechanismNotSupportedError(Exception):
    """The algorithm name is unknown to the library (oqs.py:209-215)."""

    def __init__(self, alg_name: str) -> None:
        self.alg_name = alg_name
        self.message = f"{alg_name} is not supported by OQS"
        super().__init__(self.message)


class MechanismNotEnabledError(MechanismNotSupportedError):
    """Known to the library but without an implementation (oqs.py:218-224)."""

    def __init__(self, alg_name: str) -> None:
        super().__init__(alg_name)
        self.message = f"{alg_name} is supported but not enabled by OQS"
        self.args = (self.message,)


def _names() -> tuple[str, ...]:
    return tuple(LIB.OQS_KEM_alg_identifier(i).decode() for i in range(LIB.OQS_KEM_alg_count()))


_SUPPORTED = _names()
_ENABLED = tuple(n for n in _SUPPORTED if LIB.OQS_KEM_alg_is_enabled(n.encode()))


def get_supported_kem_mechanisms() -> tuple[str, ...]:
    return _SUPPORTED


def get_enabled_kem_mechanisms() -> tuple[str, ...]:
    return _ENABLED


def is_kem_enabled(alg_name: str) -> bool:
    return bool(LIB.OQS_KEM_alg_is_enabled(alg_name.encode()))


_SIZES: dict = {}


def kem_sizes(alg_name: str) -> dict:
    # constants per mechanism, read from the library once (the reference's call pattern builds a
    # new KeyEncapsulation per encaps / decaps, so this sits on every single-shot call)
    hit = _SIZES.get(alg_name)
    if hit is not None:
        return dict(hit)
    out = (ct.c_size_t * 6)()
    if LIB.qrk_kem_sizes(alg_name.encode(), out) != 0:
        raise MechanismNotSupportedError(alg_name)
    keys = ("length_public_key", "length_secret_key", "length_ciphertext",
            "length_shared_secret", "length_keypair_coins", "length_encaps_coins")
    _SIZES[alg_name] = dict(zip(keys, (int(v) for v in out)))
    return dict(_SIZES[alg_name])


class _KemPrefix(ct.Structure):
    """Leading fields of the C ``OQS_KEM`` struct (include/qrkem.h), the prefix the reference's
    wrapper reads from the handle (oqs.py:241-253, 273-280)."""
    _fields_ = [("method_name", ct.c_char_p), ("alg_version", ct.c_char_p),
                ("claimed_nist_level", ct.c_ubyte), ("ind_cca", ct.c_ubyte),
                ("length_public_key", ct.c_size_t), ("length_secret_key", ct.c_size_t),
                ("length_ciphertext", ct.c_size_t), ("length_shared_secret", ct.c_size_t)]


def _fixed(data: Union[bytes, bytearray, memoryview], size: int) -> ct.Array:
    # ctypes.create_string_buffer(init, size) semantics (oqs.py:294-297, 338-341)
    return ct.create_string_buffer(bytes(data), size)


_ATTRS: dict = {}  # mechanism -> the handle struct's fields (constant per mechanism)


class KeyEncapsulation:
    """One KEM mechanism; mirrors ``oqs.KeyEncapsulation`` (oqs.py:227-393)."""

    def __init__(self, alg_name: str, secret_key: Union[bytes, None] = None) -> None:
        self.alg_name = alg_name
        if alg_name not in _ENABLED:
            if alg_name in _SUPPORTED:
                raise MechanismNotEnabledError(alg_name)
            raise MechanismNotSupportedError(alg_name)
        self._kem = LIB.OQS_KEM_new(alg_name.encode())
        if not self._kem:
            raise RuntimeError(f"OQS_KEM_new({alg_name}) failed: {last_error()}")
        # every attribute comes from the handle's struct, as oqs.py:273-280 reads it; the struct is
        # the same for every handle of a mechanism, so it is read once per mechanism (the reference's
        # call pattern builds a new object per encaps / decaps: ~3 us of ctypes field reads each)
        attrs = _ATTRS.get(alg_name)
        if attrs is None:
            k = ct.cast(self._kem, ct.POINTER(_KemPrefix)).contents
            sz = kem_sizes(alg_name)
            attrs = {
                "_kp_coins": sz["length_keypair_coins"],
                "_enc_coins": sz["length_encaps_coins"],
                "method_name": k.method_name,
                "alg_version": k.alg_version,
                "claimed_nist_level": int(k.claimed_nist_level),
                "ind_cca": int(k.ind_cca),
                "length_public_key": int(k.length_public_key),
                "length_secret_key": int(k.length_secret_key),
                "length_ciphertext": int(k.length_ciphertext),
                "length_shared_secret": int(k.length_shared_secret),
            }
            _ATTRS[alg_name] = attrs
        self.__dict__.update(attrs)
        self.details = {
            "name": alg_name,
            "version": self.alg_version.decode(),
            "claimed_nist_level": int(self.claimed_nist_level),
            "is_ind_cca": True,
            "length_public_key": self.length_public_key,
            "length_secret_key": self.length_secret_key,
            "length_ciphertext": self.length_ciphertext,
            "length_shared_secret": self.length_shared_secret,
        }
        if secret_key:
            self.secret_key = _fixed(secret_key, self.length_secret_key)

    def __enter__(self) -> "KeyEncapsulation":
        return self

    def __exit__(self, *exc) -> None:
        self.free()

    def generate_keypair(self) -> bytes:
        pk = ct.create_string_buffer(self.length_public_key)
        self.secret_key = ct.create_string_buffer(self.length_secret_key)
        if LIB.OQS_KEM_keypair(self._kem, pk, self.secret_key) != OQS_SUCCESS:
            raise RuntimeError("Can not generate keypair")
        return bytes(pk)

    def generate_keypair_derand(self, coins: bytes) -> bytes:
        """Deterministic KeyGen from explicit coins (d||z for ML-KEM, s||seedSE||z for FrodoKEM)."""
        coins = self._coins(coins, self._kp_coins, "keypair")
        pk = ct.create_string_buffer(self.length_public_key)
        self.secret_key = ct.create_string_buffer(self.length_secret_key)
        if LIB.OQS_KEM_keypair_derand(self._kem, pk, self.secret_key, bytes(coins)) != OQS_SUCCESS:
            raise RuntimeError("Can not generate keypair")
        return bytes(pk)

    @staticmethod
    def _coins(coins, want: int, what: str) -> bytes:
        # the library reads exactly `want` bytes: a shorter buffer would be read past its end
        c = bytes(coins)
        if len(c) != want:
            raise ValueError(f"{what} coins must be {want} bytes, got {len(c)}")
        return c

    def export_secret_key(self) -> bytes:
        return bytes(self.secret_key)

    def encap_secret(self, public_key: Union[bytes, bytearray]) -> tuple[bytes, bytes]:
        pk = _fixed(public_key, self.length_public_key)
        c = ct.create_string_buffer(self.length_ciphertext)
        ss = ct.create_string_buffer(self.length_shared_secret)
        if LIB.OQS_KEM_encaps(self._kem, c, ss, pk) != OQS_SUCCESS:
            raise RuntimeError("Can not encapsulate secret")
        return bytes(c), bytes(ss)

    def encap_secret_derand(self, public_key: bytes, coins: bytes) -> tuple[bytes, bytes]:
        coins = self._coins(coins, self._enc_coins, "encaps")
        pk = _fixed(public_key, self.length_public_key)
        c = ct.create_string_buffer(self.length_ciphertext)
        ss = ct.create_string_buffer(self.length_shared_secret)
        if LIB.OQS_KEM_encaps_derand(self._kem, c, ss, pk, bytes(coins)) != OQS_SUCCESS:
            raise RuntimeError("Can not encapsulate secret")
        return bytes(c), bytes(ss)

    def decap_secret(self, ciphertext: Union[bytes, bytearray]) -> bytes:
        c = _fixed(ciphertext, self.length_ciphertext)
        ss = ct.create_string_buffer(self.length_shared_secret)
        if LIB.OQS_KEM_decaps(self._kem, ss, c, self.secret_key) != OQS_SUCCESS:
            raise RuntimeError("Can not decapsulate secret")
        return bytes(ss)

    def free(self) -> None:
        if getattr(self, "secret_key", None) is not None:
            LIB.OQS_MEM_cleanse(ct.addressof(self.secret_key), self.length_secret_key)
        if self._kem:
            LIB.OQS_KEM_free(self._kem)
            self._kem = None

    def __repr__(self) -> str:
        return f"Key encapsulation mechanism: {self.alg_name}"
