"""Golden HQC vectors (tests/golden/hqc.json) -- TEST INFRASTRUCTURE.

PARITY UNPINNED against liboqs: liboqs (and its HQC KAT files) is absent offline and the
reference holds no HQC vectors.  These vectors freeze the pure-Python restatement
(oracle/py/hqc_spec.py, 2023-04-30 HQC) so that the C oracle and the GPU path are checked
against one fixed set of bytes.  Inputs per record i (deterministic):
  keypair coins = SHAKE256("qrk-bench" || LE64(seed) || LE64(2i)), first kp_coins bytes;
  encaps coins  = SHAKE256("qrk-bench" || LE64(seed) || LE64(2i+1)), first enc_coins bytes;
  tampered ct   = ct with bit (13 i + 5) mod 8|ct| flipped.
Stored: coins (hex), SHA-256 of pk / sk / ct / ss / tampered-ss, the tampered decaps return
code, and the full first 64 bytes of each output.

    python tests/golden/make_golden_hqc.py
"""
import hashlib
import json
import sys
from pathlib import Path

HERE = Path(__file__).resolve().parent
sys.path[:0] = [str(HERE.parents[1] / "oracle" / "py")]

import hqc_spec  # noqa: E402

SEED = 0x4851
RECORDS = 3


def coins(i: int, n: int) -> bytes:
    msg = b"qrk-bench" + SEED.to_bytes(8, "little") + i.to_bytes(8, "little")
    return hashlib.shake_256(msg).digest(n)


def tamper(ct: bytes, i: int) -> bytes:
    b = bytearray(ct)
    bit = (13 * i + 5) % (8 * len(b))
    b[bit // 8] ^= 1 << (bit % 8)
    return bytes(b)


def main():
    out = {}
    for alg in ("HQC-128", "HQC-192", "HQC-256"):
        s = hqc_spec.sizes(alg)
        recs = []
        for i in range(RECORDS):
            kc, ec = coins(2 * i, s["kp_coins"]), coins(2 * i + 1, s["enc_coins"])
            pk, sk = hqc_spec.keypair(alg, kc)
            ct, ss = hqc_spec.encaps(alg, pk, ec)
            ss_d, rc = hqc_spec.decaps(alg, sk, ct)
            assert ss_d == ss and rc == 0
            tss, trc = hqc_spec.decaps(alg, sk, tamper(ct, i))
            d = lambda b: hashlib.sha256(b).hexdigest()  # noqa: E731
            recs.append({"kp_coins": kc.hex(), "enc_coins": ec.hex(), "pk": d(pk), "sk": d(sk), "ct": d(ct),
                         "ss": ss.hex(), "tampered_ss": tss.hex(), "tampered_rc": trc,
                         "pk64": pk[:64].hex(), "ct64": ct[:64].hex()})
        out[alg] = {"sizes": s, "records": recs}
    (HERE / "hqc.json").write_text(json.dumps(out, indent=1) + "\n")


if __name__ == "__main__":
    main()
