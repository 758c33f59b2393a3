"""GPU: HKDF-SHA256 kernel (hkdf.hip) and the batched handshake driver
(qrk_handshake_batch) vs the oracle, through the C ABI.  Bar: byte-exact."""
import hashlib
import json

import numpy as np
import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def kdf():
    from qrkem.handshake import KeyDerivation
    return KeyDerivation(device=0)


def test_rfc5869_vectors_on_gpu(kdf):
    from test_handshake_oracle import RFC5869
    for ikm, salt, info, L, _prk, okm in RFC5869:
        out = kdf.derive(np.frombuffer(ikm, np.uint8).reshape(1, -1), info, L, salt=salt or None)
        assert out[0].tobytes().hex() == okm


@pytest.mark.parametrize("ikm_len,L,salt_len", [(32, 32, 0), (16, 16, 0), (24, 24, 13), (32, 33, 64),
                                                (32, 100, 65), (1, 1, 200), (32, 8160, 0)])
def test_hkdf_ragged_infos_match_oracle(kdf, ikm_len, L, salt_len):
    import oracle as orc
    rng = np.random.default_rng(ikm_len * 1000 + L + salt_len)
    n = 37 if L < 1000 else 5
    ikm = rng.integers(0, 256, (n, ikm_len), dtype=np.uint8)
    infos = [rng.integers(0, 256, int(rng.integers(0, 300)), dtype=np.uint8).tobytes() for _ in range(n)]
    infos[0] = b""
    salt = rng.integers(0, 256, salt_len, dtype=np.uint8).tobytes() or None
    dev = kdf.derive(torch.from_numpy(ikm).cuda(), infos, L, salt=salt)
    torch.cuda.synchronize()
    ref = orc.batch_hkdf(ikm, infos, L, salt=salt)
    assert np.array_equal(dev.cpu().numpy(), ref)


def test_hkdf_shared_info_large_batch(kdf):
    import oracle as orc
    from qrkem.handshake import protocol_info
    info = protocol_info("b" * 36, "a" * 36, "AES-256-GCM")
    n = 70000
    ikm = torch.randint(0, 256, (n, 32), dtype=torch.uint8, device="cuda")
    out = kdf.derive(ikm, info, 32).cpu().numpy()
    h = ikm.cpu().numpy()
    idx = list(range(0, n, 997)) + [n - 1]
    ref = orc.batch_hkdf(np.ascontiguousarray(h[idx]), [info] * len(idx), 32)
    assert np.array_equal(out[idx], ref)


@pytest.mark.parametrize("case", range(4))
def test_handshake_driver_matches_golden(golden_dir, case):
    from make_golden_handshake import CASES, inputs
    from qrkem.handshake import HandshakeDriver
    alg, n, sym = CASES[case]
    g = json.loads((golden_dir / "handshake.json").read_text())[f"{alg}|{n}|{sym}"]
    kpi, kpr, en, infos = inputs(alg, n, sym)
    drv = HandshakeDriver(alg, symmetric_name=sym)
    out = drv.run(infos, coins_kp_initiator=kpi, coins_kp_responder=kpr, coins_encaps=en)
    torch.cuda.synchronize()
    got = {"pk_i": out.pk_initiator, "pk_r": out.pk_responder, "ct": out.ciphertext, "key_i": out.key_initiator,
           "key_r": out.key_responder}
    for k, t in got.items():
        assert hashlib.sha256(t.cpu().numpy().tobytes()).hexdigest() == g["digests"][k], k
    assert bool((out.agree == 1).all())


def test_handshake_driver_multi_chunk_random_coins():
    """OS-CSPRNG coins, batch larger than one chunk: both sides must agree everywhere."""
    from qrkem.handshake import HandshakeDriver
    drv = HandshakeDriver("ML-KEM-768", chunk=4096)
    n = 10000
    infos = [drv.info_for(f"peer-{i}", "server", ) for i in range(n)]
    out = drv.run(infos)
    torch.cuda.synchronize()
    assert int(out.agree.sum()) == n
    assert torch.equal(out.key_initiator, out.key_responder)
    assert not torch.equal(out.key_initiator[0], out.key_initiator[1])


def test_key_derivation_host_inputs(kdf):
    import hkdf_spec
    ss = [bytes(range(32)), bytes(range(32, 64))]
    info = hkdf_spec.protocol_info("x", "y", "ChaCha20-Poly1305")
    out = kdf.derive(ss, [info, info], 32)
    for i in range(2):
        assert out[i].tobytes() == hkdf_spec.hkdf_sha256(ss[i], info, 32)


@pytest.mark.parametrize("alg,n,chunk", [("ML-KEM-512", 3000, 2048), ("ML-KEM-768", 3000, 2048),
                                         ("ML-KEM-1024", 3000, 2048), ("ML-KEM-768", 1089, 1088)])
def test_handshake_driver_expanded_key_reuse_matches_oracle(alg, n, chunk):
    """Batched ML-KEM chunks (> 1024 handshakes) keep the initiator's sampled matrix A_hat from its
    KeyGen (messaging.py:590) for its Decaps (:1038) instead of re-running SampleNTT; the last chunk
    (952, or a single handshake) runs the one-launch kernels without reuse; 1088 is the first
    batched chunk size, a ragged 64-handshake tile.  Every output byte-exact vs the oracle's
    handshake (a wrong A_hat would re-encrypt differently and select the implicit-rejection key)."""
    import oracle as orc
    import hkdf_spec
    from make_golden_handshake import node_id
    from qrkem.handshake import HandshakeDriver
    sym = "AES-256-GCM"
    s = orc.sizes(alg)
    kp, enc = s["keypair_coins"], s["encaps_coins"]
    coins = orc.bench_coins(n, 2 * kp + enc, seed=0xA11 + kp)
    kpi, kpr, en = (np.ascontiguousarray(coins[:, a:b]) for a, b in ((0, kp), (kp, 2 * kp), (2 * kp, 2 * kp + enc)))
    infos = [hkdf_spec.protocol_info(node_id(b"a", i), node_id(b"b", i), sym) for i in range(n)]
    drv = HandshakeDriver(alg, symmetric_name=sym, chunk=chunk)
    out = drv.run(infos, coins_kp_initiator=kpi, coins_kp_responder=kpr, coins_encaps=en)
    torch.cuda.synchronize()
    want = orc.batch_handshake(alg, kpi, kpr, en, infos, hkdf_spec.SYMMETRIC_KEY_SIZE[sym])
    got = (out.pk_initiator, out.pk_responder, out.ciphertext, out.key_initiator, out.key_responder)
    for name, g, w in zip(("pk_i", "pk_r", "ct", "key_i", "key_r"), got, want):
        assert np.array_equal(g.cpu().numpy(), w), name
    assert bool((out.agree == 1).all())
