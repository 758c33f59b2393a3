"""Golden handshake vectors (tests/golden/handshake.json) -- TEST INFRASTRUCTURE.

Inputs per handshake i (deterministic, no reference code involved):
  coins = SHAKE256("qrk-bench" || LE64(seed) || LE64(i)) (the bench derivation), split as
  initiator KeyGen coins | responder KeyGen coins | Encaps coins;
  node ids = UUID-formatted strings from SHA-256("node-a"/"node-b" || LE64(i)) (the reference
  uses str(uuid.uuid4()), networking/node_identity.py:78), info per messaging.py:364-367.
Outputs: the C oracle's batched handshake (orc_handshake_batch), whose HKDF is pinned by
RFC 5869 and whose KEMs are pinned by tests/golden/kat_*.json.  Stored as SHA-256 digests
of each output array plus the full first record.

    python tests/golden/make_golden_handshake.py
"""
import hashlib
import json
import sys
from pathlib import Path

HERE = Path(__file__).resolve().parent
sys.path[:0] = [str(HERE.parents[1] / "oracle"), str(HERE.parents[1] / "oracle" / "py")]

import numpy as np  # noqa: E402

import hkdf_spec  # noqa: E402
import oracle as orc  # noqa: E402

CASES = [("ML-KEM-768", 64, "AES-256-GCM"), ("ML-KEM-512", 16, "ChaCha20-Poly1305"),
         ("ML-KEM-1024", 16, "AES-256-GCM"), ("FrodoKEM-640-SHAKE", 4, "AES-256-GCM")]
SEED = 0x4A5D


def node_id(tag: bytes, i: int) -> str:
    h = hashlib.sha256(tag + i.to_bytes(8, "little")).hexdigest()
    return f"{h[:8]}-{h[8:12]}-4{h[13:16]}-a{h[17:20]}-{h[20:32]}"


def inputs(alg: str, n: int, sym: str):
    s = orc.sizes(alg)
    kp, enc = s["keypair_coins"], s["encaps_coins"]
    total = 2 * kp + enc
    width = (total + 7) // 8 * 8
    coins = orc.bench_coins(n, width, seed=SEED)
    kpi = np.ascontiguousarray(coins[:, :kp])
    kpr = np.ascontiguousarray(coins[:, kp:2 * kp])
    en = np.ascontiguousarray(coins[:, 2 * kp:total])
    infos = [hkdf_spec.protocol_info(node_id(b"node-a", i), node_id(b"node-b", i), sym) for i in range(n)]
    return kpi, kpr, en, infos


def handshake_case(alg: str, n: int, sym: str):
    kpi, kpr, en, infos = inputs(alg, n, sym)
    outs = orc.batch_handshake(alg, kpi, kpr, en, infos, hkdf_spec.SYMMETRIC_KEY_SIZE[sym])
    names = ("pk_i", "pk_r", "ct", "key_i", "key_r")
    digests = {k: hashlib.sha256(v.tobytes()).hexdigest() for k, v in zip(names, outs)}
    first = {"info": infos[0].decode(), "key_i": outs[3][0].tobytes().hex(), "key_r": outs[4][0].tobytes().hex(),
             "ct_sha256": hashlib.sha256(outs[2][0].tobytes()).hexdigest()}
    return digests, first


def main():
    out = {}
    for alg, n, sym in CASES:
        d, f = handshake_case(alg, n, sym)
        out[f"{alg}|{n}|{sym}"] = {"digests": d, "first": f}
    (HERE / "handshake.json").write_text(json.dumps(out, indent=1) + "\n")


if __name__ == "__main__":
    main()
