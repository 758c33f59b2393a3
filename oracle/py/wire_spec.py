"""Wire-format oracle -- TEST INFRASTRUCTURE ONLY.

The reference encodes KEM payloads with the standard library itself:
``base64.b64encode(public_key).decode()`` (quantum_resistant_p2p/app/messaging.py:607,
:852-853) and decodes them with ``base64.b64decode`` (:829).  The oracle is that same call
(RFC 4648 section 4); strict decoding (``validate=True`` plus a length check) is the contract
of the batched decoder, which rejects instead of skipping non-alphabet bytes.
"""
from __future__ import annotations

import base64
import binascii

import numpy as np


def encode_records(data: np.ndarray) -> np.ndarray:
    rows = [base64.b64encode(r.tobytes()) for r in data]
    return np.frombuffer(b"".join(rows), np.uint8).reshape(len(rows), -1) if rows else np.zeros((0, 0), np.uint8)


def decode_record(text: bytes, out_len: int):
    """bytes or None (malformed: outside the alphabet, bad padding, or wrong length)."""
    try:
        b = base64.b64decode(text, validate=True)
    except (binascii.Error, ValueError):
        return None
    return b if len(b) == out_len else None
