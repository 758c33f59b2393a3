"""qrkem -- MI355X-native batched post-quantum key exchange.

Host-side mirror of the reference's KEM path (``quantum_resistant_p2p/crypto/
key_exchange.py`` + ``vendor/oqs.py``) over ``libqrkem.so`` (hand-written HIP
for gfx950).  Importing this package loads the library and raises
``RuntimeError`` if it is missing: there is no CPU fallback.
"""
from ._native import LIB, LIB_PATH, last_error  # noqa: F401
from . import oqs  # noqa: F401
from .algorithm_base import CryptoAlgorithm  # noqa: F401
from .key_exchange import (  # noqa: F401
    FrodoKEMKeyExchange,
    HQCKeyExchange,
    KeyExchangeAlgorithm,
    KyberKeyExchange,
    MLKEMKeyExchange,
)


def device_count() -> int:
    return int(LIB.qrk_device_count())
