"""HKDF-SHA256 (RFC 5869) and the protocol info string -- TEST INFRASTRUCTURE ONLY.

Pure-Python restatement of the key derivation the reference performs after each key
exchange, ``SecureMessaging._derive_symmetric_key``
(quantum_resistant_p2p/app/messaging.py:350-382)::

    node_ids = sorted([self.node.node_id, peer_id])                       # :364
    info = f"quantum_resistant_p2p-v1-{node_ids[0]}-{node_ids[1]}-{self.symmetric.name}".encode()  # :367
    HKDF(algorithm=hashes.SHA256(), length=key_size, salt=None, info=info).derive(shared_secret)  # :369-374

The reference takes HKDF from the ``cryptography`` package, which is not installed in this
image; RFC 5869 is restated here on ``hashlib.sha256`` (FIPS 180-4) and pinned by the RFC's
own SHA-256 test cases 1-3 (tests/test_handshake_oracle.py).
"""
from __future__ import annotations

import hashlib

HASH_LEN = 32
BLOCK = 64


def hmac_sha256(key: bytes, msg: bytes) -> bytes:
    """RFC 2104: H((K0 ^ opad) || H((K0 ^ ipad) || msg))."""
    if len(key) > BLOCK:
        key = hashlib.sha256(key).digest()
    k0 = key.ljust(BLOCK, b"\0")
    inner = hashlib.sha256(bytes(b ^ 0x36 for b in k0) + msg).digest()
    return hashlib.sha256(bytes(b ^ 0x5C for b in k0) + inner).digest()


def hkdf_extract(salt: bytes | None, ikm: bytes) -> bytes:
    """RFC 5869 section 2.2; salt None -> HashLen zero bytes."""
    return hmac_sha256(salt if salt else bytes(HASH_LEN), ikm)


def hkdf_expand(prk: bytes, info: bytes, length: int) -> bytes:
    """RFC 5869 section 2.3: T(i) = HMAC(PRK, T(i-1) || info || i)."""
    if not 0 < length <= 255 * HASH_LEN:
        raise ValueError("length must be 1..8160")
    out, t, i = b"", b"", 1
    while len(out) < length:
        t = hmac_sha256(prk, t + info + bytes([i]))
        out += t
        i += 1
    return out[:length]


def hkdf_sha256(ikm: bytes, info: bytes, length: int, salt: bytes | None = None) -> bytes:
    return hkdf_expand(hkdf_extract(salt, ikm), info, length)


def protocol_info(node_id: str, peer_id: str, symmetric_name: str) -> bytes:
    """messaging.py:364-367: sorted node ids, so both peers build the same string."""
    a, b = sorted([node_id, peer_id])
    return f"quantum_resistant_p2p-v1-{a}-{b}-{symmetric_name}".encode()


# Key sizes of the reference's symmetric ciphers (crypto/symmetric.py:70-81, 168-179)
SYMMETRIC_KEY_SIZE = {"AES-256-GCM": 32, "ChaCha20-Poly1305": 32}
