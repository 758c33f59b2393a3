"""Shape contract of the batched Python API, on CPU tensors (no kernel launch).

The C ABI takes raw pointers and indexes rows at the mechanism's fixed length, so
`qrkem.batch._check_dev` is what stops a wrong-width device tensor before launch;
the GPU side of the same contract is `test_gpu_edges.test_wrong_width_device_tensors_raise`.
"""
import pytest

torch = pytest.importorskip("torch")


def test_check_dev_accepts_exact_shape():
    from qrkem.batch import _check_dev
    t = torch.zeros((5, 1184), dtype=torch.uint8)
    assert _check_dev(t, 1184, "pk") is t
    assert _check_dev(t, 1184, "pk", 5) is t


@pytest.mark.parametrize("make", [
    lambda: torch.zeros((5, 1183), dtype=torch.uint8),           # short rows
    lambda: torch.zeros((5, 1185), dtype=torch.uint8),           # long rows
    lambda: torch.zeros((5 * 1184,), dtype=torch.uint8),         # flat
    lambda: torch.zeros((5, 1184), dtype=torch.int8),            # wrong dtype
    lambda: torch.zeros((1184, 5), dtype=torch.uint8).t(),       # non-contiguous view
    lambda: torch.zeros((4, 1184), dtype=torch.uint8),           # batch size mismatch
])
def test_check_dev_rejects(make):
    from qrkem.batch import _check_dev
    with pytest.raises(ValueError):
        _check_dev(make(), 1184, "pk", 5)
