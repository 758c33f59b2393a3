"""Test configuration: import paths and the `gpu` marker.

`-m "not gpu"` runs on CPU (oracle vs golden vectors, C-ABI load/exports,
host-side surface); `-m gpu` runs the HIP parity tests through the C ABI.
"""
import sys
from pathlib import Path

import pytest

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
