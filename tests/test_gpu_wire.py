"""GPU: batched base64 codec (wire.hip) vs the reference's own encoder (Python base64,
messaging.py:607, 829, 852-853).  Bar: byte-exact text and bytes; malformed records flagged
exactly where strict decoding (b64decode(validate=True) + length) rejects them."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu

LENGTHS = [1, 2, 3, 4, 5, 11, 12, 13, 16, 23, 24, 25, 32, 768, 800, 1088, 1184, 1568, 9616, 15744]


@pytest.fixture(scope="module")
def codec():
    from qrkem.wire import Base64Codec
    return Base64Codec(device=0)


@pytest.mark.parametrize("L", LENGTHS)
def test_encode_decode_match_python(codec, L):
    import wire_spec
    rng = np.random.default_rng(L)
    n = 37 if L < 5000 else 5
    data = rng.integers(0, 256, (n, L), dtype=np.uint8)
    txt = codec.encode(torch.from_numpy(data).cuda())
    torch.cuda.synchronize()
    assert np.array_equal(txt.cpu().numpy(), wire_spec.encode_records(data))
    back, st = codec.decode(txt, L)
    torch.cuda.synchronize()
    assert np.array_equal(back.cpu().numpy(), data)
    assert int(st.abs().sum()) == 0


def test_malformed_records_flagged(codec):
    import wire_spec
    rng = np.random.default_rng(3)
    for L in (1, 2, 3, 10, 1184):
        n = 64
        data = rng.integers(0, 256, (n, L), dtype=np.uint8)
        txt = wire_spec.encode_records(data).copy()
        W = txt.shape[1]
        for i in range(1, n, 2):  # corrupt odd records
            kind = (i // 2) % 4
            pos = int(rng.integers(0, W))
            if kind == 0:
                txt[i, pos] = ord("!")
            elif kind == 1:
                txt[i, pos] = 0xC3  # non-ASCII
            elif kind == 2:
                txt[i, min(pos, max(W - 5, 0))] = ord("=")  # padding in the middle
            else:
                txt[i, -1] = ord("A") if txt[i, -1] == ord("=") else ord("=")  # padding count
        out, st = codec.decode(torch.from_numpy(txt).cuda(), L)
        torch.cuda.synchronize()
        st, out = st.cpu().numpy(), out.cpu().numpy()
        for i in range(n):
            want = wire_spec.decode_record(txt[i].tobytes(), L)
            assert (st[i] == 0) == (want is not None), (L, i, txt[i].tobytes()[-8:])
            if want is not None:
                assert out[i].tobytes() == want


def test_large_batch_roundtrip(codec):
    n, L = 1 << 18, 1184
    data = torch.randint(0, 256, (n, L), dtype=torch.uint8, device="cuda")
    txt = codec.encode(data)
    back, st = codec.decode(txt, L)
    torch.cuda.synchronize()
    assert torch.equal(back, data) and int(st.abs().sum()) == 0
    import base64
    idx = [0, 1, n // 2, n - 1]
    h = data[idx].cpu().numpy()
    t = txt[idx].cpu().numpy()
    for a, b in zip(h, t):
        assert base64.b64encode(a.tobytes()) == b.tobytes()
