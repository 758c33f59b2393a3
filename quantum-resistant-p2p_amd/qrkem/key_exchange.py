"""Post-quantum key-exchange plugins backed by the MI355X engine.

Drop-in counterpart of ``quantum_resistant_p2p/crypto/key_exchange.py``:

* ``KeyExchangeAlgorithm`` -- abstract ``generate_keypair() -> (pk, sk)``,
  ``encapsulate(pk) -> (ct, ss)``, ``decapsulate(sk, ct) -> ss``
  (argument order private key first, ``:44``), ``key_exchange.py:19-54``;
* ``MLKEMKeyExchange(security_level=3)`` -- levels 1/3/5 -> ML-KEM-512/768/1024,
  names "ML-KEM (Level n)", ``ValueError`` for other levels, ``:57-186``.  The
  reference's Kyber fallback (``:82-99``) never triggers here because ML-KEM is
  always enabled; Kyber names are not offered (different bytes);
* ``FrodoKEMKeyExchange(security_level=3, use_aes=True)`` -- AES/SHAKE variant
  maps and cross-PRG fallback (``:312-367``), keeping the reference's naming
  quirk: ``name`` reports the *requested* PRG even after a fallback (``:369-379``);
* ``HQCKeyExchange(security_level=3)`` -- levels 1/3/5 -> HQC-128/192/256, names
  "HQC (Level n)", same constructor contract (``:189-229``).  As with liboqs, ``decapsulate``
  raises ``RuntimeError`` when the ciphertext fails HQC's re-encryption check (liboqs's
  HQC decaps returns an error there, surfaced by ``oqs.py:372-380``).

Single-handshake methods keep the reference's call pattern (a fresh mechanism
object for encaps/decaps) but every KEM operation runs on the GPU.  Added:
``generate_keypairs(n)``, ``encapsulate_batch(pks)``, ``decapsulate_batch(sks, cts)``
over ``[n, len]`` arrays (numpy on host, or torch uint8 on ``cuda``).
"""
from __future__ import annotations

import abc
import logging
from typing import Tuple

from . import oqs
from .algorithm_base import CryptoAlgorithm

logger = logging.getLogger(__name__)


class KeyExchangeAlgorithm(CryptoAlgorithm):
    @abc.abstractmethod
    def generate_keypair(self) -> Tuple[bytes, bytes]:
        ...

    @abc.abstractmethod
    def encapsulate(self, public_key: bytes) -> Tuple[bytes, bytes]:
        ...

    @abc.abstractmethod
    def decapsulate(self, private_key: bytes, ciphertext: bytes) -> bytes:
        ...


class _OQSBackedKEM(KeyExchangeAlgorithm):
    """Shared single-shot + batched plumbing (the reference repeats it per class)."""

    _family = "KEM"
    variant: str

    def _open(self) -> None:
        self.kem = oqs.KeyEncapsulation(self.variant)
        self._batch = None

    def generate_keypair(self) -> Tuple[bytes, bytes]:
        try:
            pk = self.kem.generate_keypair()
            sk = self.kem.export_secret_key()
            return pk, sk
        except Exception as exc:
            logger.error("Error generating %s keypair: %s", self._family, exc)
            raise

    def encapsulate(self, public_key: bytes) -> Tuple[bytes, bytes]:
        try:
            return oqs.KeyEncapsulation(self.variant).encap_secret(public_key)
        except Exception as exc:
            logger.error("Error during %s encapsulation: %s", self._family, exc)
            raise

    def decapsulate(self, private_key: bytes, ciphertext: bytes) -> bytes:
        try:
            return oqs.KeyEncapsulation(self.variant, private_key).decap_secret(ciphertext)
        except Exception as exc:
            logger.error("Error during %s decapsulation: %s", self._family, exc)
            raise

    # -------- batched extensions (no reference equivalent)
    @property
    def batch(self):
        if self._batch is None:
            from .batch import BatchKEM
            self._batch = BatchKEM(self.variant)
        return self._batch

    def generate_keypairs(self, n: int = None, coins=None):
        return self.batch.keypair(n=n, coins=coins)

    def encapsulate_batch(self, public_keys, coins=None):
        return self.batch.encaps(public_keys, coins=coins)

    def decapsulate_batch(self, private_keys, ciphertexts):
        return self.batch.decaps(private_keys, ciphertexts)


class MLKEMKeyExchange(_OQSBackedKEM):
    _family = "ML-KEM"
    _VARIANTS = {1: "ML-KEM-512", 3: "ML-KEM-768", 5: "ML-KEM-1024"}

    def __init__(self, security_level: int = 3):
        self.security_level = security_level
        self.kem = None
        self.variant = None
        if security_level not in self._VARIANTS:
            raise ValueError(f"Invalid security level: {security_level}. Must be 1, 3, or 5.")
        self.enabled_kems = oqs.get_enabled_kem_mechanisms()
        if self._VARIANTS[security_level] not in self.enabled_kems:
            raise ValueError(f"No ML-KEM or Kyber variant found for security level {security_level}")
        self.variant = self._VARIANTS[security_level]
        self._open()
        logger.info("Initialized ML-KEM key exchange with security level %s", security_level)

    @property
    def name(self) -> str:
        return f"ML-KEM (Level {self.security_level})"

    @property
    def display_name(self) -> str:
        return f"ML-KEM (Level {self.security_level})"

    @property
    def description(self) -> str:
        return ("ML-KEM is a module-lattice-based key encapsulation mechanism. "
                "It is one of the NIST post-quantum cryptography standards.")


class HQCKeyExchange(_OQSBackedKEM):
    _family = "HQC"
    _VARIANTS = {1: "HQC-128", 3: "HQC-192", 5: "HQC-256"}

    def __init__(self, security_level: int = 3):
        self.security_level = security_level
        self.kem = None
        self.variant = None
        if security_level not in self._VARIANTS:
            raise ValueError(f"Invalid security level: {security_level}. Must be 1, 3, or 5.")
        self.enabled_kems = oqs.get_enabled_kem_mechanisms()
        if self._VARIANTS[security_level] not in self.enabled_kems:
            raise ValueError(f"No HQC variant found for security level {security_level}")
        self.variant = self._VARIANTS[security_level]
        self._open()

    @property
    def name(self) -> str:
        return f"HQC (Level {self.security_level})"

    @property
    def display_name(self) -> str:
        return f"HQC (Level {self.security_level})"

    @property
    def description(self) -> str:
        return ("HQC (Hamming Quasi-Cyclic) is a code-based key encapsulation mechanism. "
                "It uses error-correcting codes and is based on the hardness of "
                "decoding problems.")


class FrodoKEMKeyExchange(_OQSBackedKEM):
    _family = "FrodoKEM"
    _N = {1: 640, 3: 976, 5: 1344}

    def __init__(self, security_level: int = 3, use_aes: bool = True):
        self.security_level = security_level
        self.use_aes = use_aes
        self.kem = None
        self.variant = None
        if security_level not in self._N:
            raise ValueError(f"Invalid security level: {security_level}. Must be 1, 3, or 5.")
        wanted = f"FrodoKEM-{self._N[security_level]}-{'AES' if use_aes else 'SHAKE'}"
        other = f"FrodoKEM-{self._N[security_level]}-{'SHAKE' if use_aes else 'AES'}"
        self.enabled_kems = oqs.get_enabled_kem_mechanisms()
        if wanted in self.enabled_kems:
            self.variant = wanted
        elif other in self.enabled_kems:
            self.variant = other
            logger.info("Using alternative FrodoKEM variant: %s", other)
        else:
            raise ValueError(f"No FrodoKEM variant found for security level {security_level}")
        self._open()

    @property
    def name(self) -> str:
        return f"FrodoKEM (Level {self.security_level}, {'AES' if self.use_aes else 'SHAKE'})"

    @property
    def display_name(self) -> str:
        return self.name

    @property
    def description(self) -> str:
        return ("FrodoKEM is a lattice-based key encapsulation mechanism based on "
                "the standard Learning With Errors problem. It is considered "
                "a conservative post-quantum KEM.")


# The reference re-exports ML-KEM under its pre-standard name
# (quantum_resistant_p2p/crypto/__init__.py:19).
KyberKeyExchange = MLKEMKeyExchange
