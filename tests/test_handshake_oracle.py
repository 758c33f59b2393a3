"""CPU: the HKDF-SHA256 / handshake oracle (oracle/src/hkdf.c, oracle/py/hkdf_spec.py).

Pins HKDF against RFC 5869 Appendix A test cases 1-3 (the SHA-256 ones) and SHA-256
against hashlib, checks the protocol info string of messaging.py:364-367, and checks the
C handshake driver against the committed golden digests (tests/golden/handshake.json,
made by tests/golden/make_golden_handshake.py) and against the single-record calls.
"""
import hashlib
import json

import numpy as np
import pytest

import hkdf_spec
import oracle as orc

# RFC 5869 Appendix A.1-A.3: (IKM, salt, info, L, PRK, OKM)
RFC5869 = [
    (bytes([0x0B] * 22), bytes(range(0x00, 0x0D)), bytes(range(0xF0, 0xFA)), 42,
     "077709362c2e32df0ddc3f0dc47bba6390b6c73bb50f9c3122ec844ad7c2b3e5",
     "3cb25f25faacd57a90434f64d0362f2a2d2d0a90cf1a5a4c5db02d56ecc4c5bf34007208d5b887185865"),
    (bytes(range(0x00, 0x50)), bytes(range(0x60, 0xB0)), bytes(range(0xB0, 0x100)), 82,
     "06a6b88c5853361a06104c9ceb35b45cef760014904671014a193f40c15fc244",
     "b11e398dc80327a1c8e7f78c596a49344f012eda2d4efad8a050cc4c19afa97c59045a99cac7827271cb41c65e590e09"
     "da3275600c2f09b8367793a9aca3db71cc30c58179ec3e87c14c01d5c1f3434f1d87"),
    (bytes([0x0B] * 22), b"", b"", 42,
     "19ef24a32c717b167f33a91d6f648bdf96596776afdb6377ac434c1c293ccb04",
     "8da4e775a563c18f715f802a063c5a31b8a11f5c5ee1879ec3454e5f3c738d2d9d201395faa4b61a96c8"),
]


@pytest.mark.parametrize("case", range(3))
def test_rfc5869_vectors(case):
    ikm, salt, info, L, prk, okm = RFC5869[case]
    assert hkdf_spec.hkdf_extract(salt, ikm).hex() == prk
    assert hkdf_spec.hkdf_sha256(ikm, info, L, salt).hex() == okm
    assert orc.hkdf_sha256(ikm, info, L, salt).hex() == okm


def test_sha256_vs_hashlib():
    rng = np.random.default_rng(5)
    for n in (0, 1, 55, 56, 63, 64, 65, 119, 120, 200, 1000):
        m = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        assert orc.sha256(m) == hashlib.sha256(m).digest()


def test_hkdf_c_vs_python_edge_cases():
    rng = np.random.default_rng(6)
    for ikm_len, info_len, L, salt_len in [(32, 110, 32, 0), (16, 0, 1, 0), (24, 300, 33, 13), (32, 55, 64, 64),
                                           (32, 56, 100, 65), (0, 1, 8160, 200)]:
        ikm = rng.integers(0, 256, ikm_len, dtype=np.uint8).tobytes()
        info = rng.integers(0, 256, info_len, dtype=np.uint8).tobytes()
        salt = rng.integers(0, 256, salt_len, dtype=np.uint8).tobytes() or None
        assert orc.hkdf_sha256(ikm, info, L, salt) == hkdf_spec.hkdf_sha256(ikm, info, L, salt)


def test_protocol_info_is_order_independent():
    a, b = "9f1c0f0e-3a6b-4a4e-9d1e-2f3a4b5c6d7e", "1a2b3c4d-5e6f-4711-8899-aabbccddeeff"
    info = hkdf_spec.protocol_info(a, b, "AES-256-GCM")
    assert info == hkdf_spec.protocol_info(b, a, "AES-256-GCM")
    assert info == f"quantum_resistant_p2p-v1-{b}-{a}-AES-256-GCM".encode()
    from qrkem.handshake import protocol_info
    assert protocol_info(a, b, "ChaCha20-Poly1305") == hkdf_spec.protocol_info(a, b, "ChaCha20-Poly1305")


def test_batch_hkdf_matches_single():
    rng = np.random.default_rng(7)
    ikm = rng.integers(0, 256, (50, 32), dtype=np.uint8)
    infos = [rng.integers(0, 256, int(rng.integers(0, 200)), dtype=np.uint8).tobytes() for _ in range(50)]
    out = orc.batch_hkdf(ikm, infos, 32, threads=4)
    for i in range(50):
        assert out[i].tobytes() == hkdf_spec.hkdf_sha256(ikm[i].tobytes(), infos[i], 32)


def test_handshake_golden(golden_dir):
    from make_golden_handshake import CASES, handshake_case
    g = json.loads((golden_dir / "handshake.json").read_text())
    for alg, n, sym in CASES:
        rec = g[f"{alg}|{n}|{sym}"]
        digests, first = handshake_case(alg, n, sym)
        assert digests == rec["digests"], alg
        assert first == rec["first"], alg


def test_handshake_driver_vs_single_calls():
    from make_golden_handshake import inputs
    alg = "ML-KEM-512"
    kpi, kpr, enc, infos = inputs(alg, 3, "ChaCha20-Poly1305")
    pk_i, pk_r, c, key_i, key_r = orc.batch_handshake(alg, kpi, kpr, enc, infos, 32, threads=2)
    assert np.array_equal(key_i, key_r)
    for i in range(3):
        pk, sk = orc.keypair(alg, kpi[i].tobytes())
        assert pk == pk_i[i].tobytes()
        ct_, ss = orc.encaps(alg, pk, enc[i].tobytes())
        assert ct_ == c[i].tobytes()
        assert hkdf_spec.hkdf_sha256(ss, infos[i], 32) == key_r[i].tobytes()
        assert orc.keypair(alg, kpr[i].tobytes())[0] == pk_r[i].tobytes()


def test_wire_oracle_is_python_base64():
    import base64
    import wire_spec
    rng = np.random.default_rng(9)
    d = rng.integers(0, 256, (4, 1184), dtype=np.uint8)
    enc = wire_spec.encode_records(d)
    assert enc.shape == (4, 1580)
    for i in range(4):
        assert enc[i].tobytes() == base64.b64encode(d[i].tobytes())
        assert wire_spec.decode_record(enc[i].tobytes(), 1184) == d[i].tobytes()
    assert wire_spec.decode_record(b"QUJD!A==", 4) is None
    assert wire_spec.decode_record(b"QUJD", 2) is None
