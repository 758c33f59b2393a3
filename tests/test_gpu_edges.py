"""GPU: edge cases of every batched entry point -- empty batches (n = 0) are no-ops that
return 0, bad arguments fail loudly with OQS_ERROR semantics (-1 + message), and outputs of
1-record batches match the single-shot OQS calls."""
import ctypes as ct

import numpy as np
import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu


def test_empty_batches_are_noops():
    from qrkem._native import LIB
    from qrkem.batch import BatchKEM
    from qrkem.handshake import HandshakeDriver, KeyDerivation
    from qrkem.wire import Base64Codec
    eng = BatchKEM("ML-KEM-768")
    z = torch.empty((0, 1), dtype=torch.uint8, device="cuda")
    s = eng._stream()
    assert LIB.qrk_kem_keypair_batch(eng._ctx, b"ML-KEM-768", 0, None, None, None, s) == 0
    assert LIB.qrk_kem_encaps_batch(eng._ctx, b"ML-KEM-768", 0, None, None, None, None, None, s) == 0
    assert LIB.qrk_kem_decaps_batch(eng._ctx, b"ML-KEM-768", 0, None, None, None, s) == 0
    kdf = KeyDerivation()
    out = kdf.derive(torch.empty((0, 32), dtype=torch.uint8, device="cuda"), b"info", 32)
    assert tuple(out.shape) == (0, 32)
    codec = Base64Codec()
    assert tuple(codec.encode(torch.empty((0, 1184), dtype=torch.uint8, device="cuda")).shape) == (0, 1580)
    drv = HandshakeDriver("ML-KEM-512")
    r = drv.run([], n=0)
    assert tuple(r.key_initiator.shape) == (0, 32)
    del z


def test_bad_arguments_fail_loudly():
    from qrkem._native import LIB, last_error
    from qrkem.handshake import KeyDerivation
    kdf = KeyDerivation()
    x = torch.zeros((2, 32), dtype=torch.uint8, device="cuda")
    with pytest.raises(RuntimeError):
        kdf.derive(x, b"i", 0)
    with pytest.raises(RuntimeError):
        kdf.derive(x, b"i", 255 * 32 + 1)
    h = ct.c_void_p()
    assert LIB.qrk_ctx_create(ct.byref(h), 0) == 0
    assert LIB.qrk_kem_keypair_batch(h, b"Kyber768", 1, None, None, None, None) == -1
    assert "unsupported" in last_error()
    assert LIB.qrk_kem_keypair_batch(h, b"BIKE-L1", 1, None, None, None, None) == -1
    assert "unsupported" in last_error()
    LIB.qrk_ctx_destroy(h)


@pytest.mark.parametrize("alg", ["ML-KEM-768", "FrodoKEM-976-SHAKE", "HQC-128"])
def test_wrong_width_device_tensors_raise(alg):
    """Device inputs are shape-checked like host ones (a wrong row width would make the
    kernels read past the tensor): ValueError, as the reference raises on a too-long
    input (oqs.py:341-347)."""
    from qrkem.batch import BatchKEM
    eng = BatchKEM(alg, device=0)
    d = lambda *s: torch.zeros(s, dtype=torch.uint8, device="cuda")  # noqa: E731
    with pytest.raises(ValueError):
        eng.keypair(coins=d(3, eng.kp_coins + 8))
    pk, sk = eng.keypair(coins=d(3, eng.kp_coins))
    with pytest.raises(ValueError):
        eng.encaps(pk[:, 1:].contiguous())
    with pytest.raises(ValueError):
        eng.encaps(pk, coins=d(2, eng.enc_coins))
    c, _ = eng.encaps(pk, coins=d(3, eng.enc_coins))
    with pytest.raises(ValueError):
        eng.decaps(sk, c[:2].contiguous())
    with pytest.raises(ValueError):
        eng.decaps(sk.view(torch.int8), c)
    with pytest.raises(ValueError):
        eng.tamper(d(3, eng.ct_len - 1), seed=1, mode=1)


@pytest.mark.parametrize("alg", ["ML-KEM-512", "ML-KEM-1024", "FrodoKEM-976-AES"])
def test_batch_of_one_matches_single_shot(alg):
    import oracle as orc
    from qrkem import oqs
    from qrkem.batch import BatchKEM
    s = orc.sizes(alg)
    coins = orc.bench_coins(1, (s["keypair_coins"] + s["encaps_coins"] + 7) // 8 * 8, seed=77)
    kc = np.ascontiguousarray(coins[:, :s["keypair_coins"]])
    ec = np.ascontiguousarray(coins[:, s["keypair_coins"]:s["keypair_coins"] + s["encaps_coins"]])
    eng = BatchKEM(alg)
    pk, sk = eng.keypair(coins=kc)            # host arrays -> host path
    c, ss = eng.encaps(pk, coins=ec)
    k = oqs.KeyEncapsulation(alg)
    pk1 = k.generate_keypair_derand(kc[0].tobytes())
    assert pk1 == pk[0].tobytes() and k.export_secret_key() == sk[0].tobytes()
    c1, ss1 = k.encap_secret_derand(pk1, ec[0].tobytes())
    assert c1 == c[0].tobytes() and ss1 == ss[0].tobytes()
    assert oqs.KeyEncapsulation(alg, sk[0].tobytes()).decap_secret(c1) == ss1
