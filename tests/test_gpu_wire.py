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


@pytest.mark.parametrize("L", [1, 2, 3, 5])
def test_tight_hipmalloc_buffers(codec, L):
    """records shorter than a 12-byte (16-character) chunk must not be loaded past the
    end of the input.  The input here is a bare hipMalloc of exactly n*L bytes (n*IL characters),
    not a torch tensor whose caching allocator pads the block, so the last records' chunks end at
    the allocation's last byte."""
    import ctypes as ct
    import wire_spec
    from qrkem._native import LIB
    hip = ct.CDLL("libamdhip64.so")
    n = 8191  # odd count: the last record's chunk is not 4-byte aligned for every L
    rng = np.random.default_rng(100 + L)
    data = rng.integers(0, 256, (n, L), dtype=np.uint8)
    want_txt = wire_spec.encode_records(data)
    IL = want_txt.shape[1]
    pin, ptxt = ct.c_void_p(), ct.c_void_p()
    assert hip.hipMalloc(ct.byref(pin), ct.c_size_t(n * L)) == 0
    assert hip.hipMalloc(ct.byref(ptxt), ct.c_size_t(n * IL)) == 0
    try:
        assert hip.hipMemcpy(pin, data.ctypes.data_as(ct.c_void_p), ct.c_size_t(n * L), 1) == 0
        assert hip.hipMemcpy(ptxt, want_txt.ctypes.data_as(ct.c_void_p), ct.c_size_t(n * IL), 1) == 0
        txt = torch.empty((n, IL), dtype=torch.uint8, device="cuda")
        back = torch.empty((n, L), dtype=torch.uint8, device="cuda")
        st = torch.zeros((n,), dtype=torch.int32, device="cuda")
        torch.cuda.synchronize()
        s = ct.c_void_p(torch.cuda.current_stream().cuda_stream)
        assert LIB.qrk_base64_encode_batch(codec._ctx, n, pin, L, ct.c_void_p(txt.data_ptr()), s) == 0
        assert LIB.qrk_base64_decode_batch(codec._ctx, n, ptxt, L, ct.c_void_p(back.data_ptr()),
                                           ct.c_void_p(st.data_ptr()), s) == 0
        torch.cuda.synchronize()
        assert np.array_equal(txt.cpu().numpy(), want_txt)
        assert np.array_equal(back.cpu().numpy(), data)
        assert int(st.abs().sum()) == 0
    finally:
        hip.hipFree(pin)
        hip.hipFree(ptxt)
