"""Test configuration: import paths and the `gpu` marker.

`-m "not gpu"` runs on CPU (oracle vs golden vectors, C-ABI load/exports,
host-side surface); `-m gpu` runs the HIP parity tests through the C ABI.
"""
import os
import sys
from pathlib import Path

import pytest

# The GPU tests run with the batched ML-KEM sampled-matrix region poisoned (0xFF) before every
# Encaps / Decaps, so a kernel that read an entry its call had not written yet would produce
# wrong bytes instead of silently reusing the previous call's identical matrix (mlkem.hip,
# debug_poison; read once, when the library first runs a batched ML-KEM call).
os.environ.setdefault("QRK_DEBUG_POISON", "1")

ROOT = Path(__file__).resolve().parents[1]
for p in (ROOT / "quantum-resistant-p2p_amd", ROOT / "oracle", ROOT / "oracle" / "py", ROOT / "tests" / "golden", ROOT):
    if str(p) not in sys.path:
        sys.path.insert(0, str(p))

GOLDEN = ROOT / "tests" / "golden"


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP kernels)")


@pytest.fixture(scope="session")
def golden_dir():
    return GOLDEN


def gpu_available() -> bool:
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False
