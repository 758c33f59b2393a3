#!/usr/bin/env python3
"""Generate tests/golden/*.json with the pure-Python restatements (oracle/py).

Run from the repo root:  python tests/golden/make_golden.py
(~2 minutes; the fixtures are committed, so tests never re-run this.)

Fixtures:
  kat_mlkem.json  NIST-KAT-DRBG handshakes (PQCgenKAT_kem procedure: entropy
                  0x00..0x2F, seed_i = i-th 48-byte draw, per record reseed,
                  KeyGen = one randombytes(64), Encaps = one randombytes(32)):
                  SHA-256 over the concatenation of every record's pk/sk/ct/ss,
                  plus the first records in full.  1024 records for ML-KEM-768
                  (BASELINE.json configs[0]), 100 for ML-KEM-512/1024.
  kat_frodo.json  the same procedure for FrodoKEM-640/976/1344-SHAKE (10 records)
                  and FrodoKEM-640/976/1344-AES (1 record each; pure-Python AES is slow;
                  976/1344-AES were appended with kat_records(F, alg, 1, ...) directly).
  tampered.json   ML-KEM-768 decapsulation of bit-flipped ciphertexts
                  (implicit rejection K_bar = J(z || c')).
  coins.json      bench coin derivation SHAKE256("qrk-bench"||LE64 seed||LE64 i).

Parity status: these vectors pin the C oracle and the HIP kernels to an
independent restatement of FIPS 203 / FrodoKEM round 3; they are NOT liboqs
KATs (liboqs is absent from the reference tree and offline), except that the
DRBG seeds reproduce the published NIST KAT seeds (tests/test_oracle.py).
"""
from __future__ import annotations

import hashlib
import json
import sys
from pathlib import Path

HERE = Path(__file__).resolve().parent
sys.path.insert(0, str(HERE.parents[1] / "oracle" / "py"))

import frodo_spec as F  # noqa: E402
import kat_drbg as D  # noqa: E402
import mlkem_spec as M  # noqa: E402


def kat_records(mod, alg, count, kp_len, enc_len):
    seeds = D.kat_seeds(count)
    h = {k: hashlib.sha256() for k in ("pk", "sk", "ct", "ss")}
    full = []
    for i, seed in enumerate(seeds):
        drbg = D.KatDrbg(seed)
        kc = drbg.randombytes(kp_len)
        ec = drbg.randombytes(enc_len)
        pk, sk = mod.keypair_derand(alg, kc)
        ct, ss = mod.encaps_derand(alg, pk, ec)
        ss2 = mod.decaps(alg, sk, ct)
        assert ss2 == ss, (alg, i)
        for k, v in (("pk", pk), ("sk", sk), ("ct", ct), ("ss", ss)):
            h[k].update(v)
        if i < 3:
            full.append({"count": i, "seed": seed.hex(), "pk_sha256": hashlib.sha256(pk).hexdigest(),
                         "sk_sha256": hashlib.sha256(sk).hexdigest(), "ct": ct.hex() if len(ct) < 2000 else None,
                         "ct_sha256": hashlib.sha256(ct).hexdigest(), "ss": ss.hex(),
                         "pk": pk.hex() if len(pk) < 2000 else None})
    return {"alg": alg, "count": count, "kp_coins": kp_len, "enc_coins": enc_len,
            "digests": {k: v.hexdigest() for k, v in h.items()}, "records": full}


def main():
    out = {}
    for alg, count in (("ML-KEM-768", 1024), ("ML-KEM-512", 100), ("ML-KEM-1024", 100)):
        out[alg] = kat_records(M, alg, count, 64, 32)
        print(alg, "done", file=sys.stderr)
    (HERE / "kat_mlkem.json").write_text(json.dumps(out, indent=1))

    fr = {}
    for alg, count in (("FrodoKEM-640-SHAKE", 10), ("FrodoKEM-976-SHAKE", 10), ("FrodoKEM-1344-SHAKE", 10),
                       ("FrodoKEM-640-AES", 1)):
        s = F.sizes(alg)
        fr[alg] = kat_records(F, alg, count, s["keypair_coins"], s["encaps_coins"])
        print(alg, "done", file=sys.stderr)
    (HERE / "kat_frodo.json").write_text(json.dumps(fr, indent=1))

    alg = "ML-KEM-768"
    pk, sk = M.keypair_derand(alg, bytes(range(64)))
    ct, ss = M.encaps_derand(alg, pk, bytes(range(64, 96)))
    cases = []
    for bit in (0, 7, 8 * 640 + 3, 8 * 1087 + 7, 8 * 960):  # in c1, c1 end region, c2
        bad = bytearray(ct)
        bad[bit // 8] ^= 1 << (bit % 8)
        cases.append({"bit": bit, "ss": M.decaps(alg, sk, bytes(bad)).hex()})
    tam = {"alg": alg, "keypair_coins": bytes(range(64)).hex(), "encaps_coins": bytes(range(64, 96)).hex(),
           "ss_valid": ss.hex(), "ct_sha256": hashlib.sha256(ct).hexdigest(), "cases": cases}
    (HERE / "tampered.json").write_text(json.dumps(tam, indent=1))

    coins = {"seed": 0x5EED, "len": 96, "items": []}
    for i in (0, 1, 4095, 1 << 20):
        m = b"qrk-bench" + (0x5EED).to_bytes(8, "little") + i.to_bytes(8, "little")
        coins["items"].append({"i": i, "coins": hashlib.shake_256(m).digest(96).hex()})
    (HERE / "coins.json").write_text(json.dumps(coins, indent=1))


if __name__ == "__main__":
    main()
