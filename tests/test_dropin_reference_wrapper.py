"""CPU: the reference's own ctypes wrapper (quantum_resistant_p2p/vendor/oqs.py)
and KEM plugins (crypto/key_exchange.py) load libqrkem.so in place of liboqs.so.

Build container only: skipped where /root/reference is absent (the GPU box).
The wrapper finds the library through its documented fallback,
$OQS_INSTALL_PATH/lib/liboqs.so (oqs.py:155-174), pointed at a temporary
symlink to libqrkem.so.  Nothing from the reference is copied.
"""
import importlib.util
import os
import sys
import types
from pathlib import Path

import pytest

REF = Path("/root/reference/quantum_resistant_p2p")
pytestmark = pytest.mark.skipif(not REF.exists(), reason="reference tree not available here")


@pytest.fixture(scope="module")
def ref_oqs(tmp_path_factory):
    import qrkem
    d = tmp_path_factory.mktemp("oqs_install")
    (d / "lib").mkdir()
    os.symlink(qrkem.LIB_PATH, d / "lib" / "liboqs.so")
    old = os.environ.get("OQS_INSTALL_PATH")
    os.environ["OQS_INSTALL_PATH"] = str(d)
    try:
        spec = importlib.util.spec_from_file_location("ref_vendor_oqs", REF / "vendor" / "oqs.py")
        mod = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(mod)
    finally:
        if old is None:
            os.environ.pop("OQS_INSTALL_PATH", None)
        else:
            os.environ["OQS_INSTALL_PATH"] = old
    return mod


def test_reference_wrapper_loads_qrkem(ref_oqs):
    assert "qrkem" in ref_oqs.oqs_version()
    enabled = ref_oqs.get_enabled_kem_mechanisms()
    assert {"ML-KEM-512", "ML-KEM-768", "ML-KEM-1024"} <= set(enabled)
    k = ref_oqs.KeyEncapsulation("ML-KEM-768")
    assert k.details["length_public_key"] == 1184
    assert k.details["length_secret_key"] == 2400
    assert k.details["length_ciphertext"] == 1088
    assert k.details["length_shared_secret"] == 32
    assert k.details["claimed_nist_level"] == 3 and k.details["is_ind_cca"]
    h = ref_oqs.KeyEncapsulation("HQC-128")
    assert (h.details["length_public_key"], h.details["length_secret_key"], h.details["length_ciphertext"],
            h.details["length_shared_secret"]) == (2249, 2305, 4433, 64)
    with pytest.raises(ref_oqs.MechanismNotSupportedError):
        ref_oqs.KeyEncapsulation("BIKE-L1")
    with pytest.raises(ref_oqs.MechanismNotSupportedError):
        ref_oqs.KeyEncapsulation("Kyber768")


def test_reference_plugins_on_qrkem(ref_oqs):
    """crypto/key_exchange.py over the reference wrapper over libqrkem.so."""
    sys.modules["oqs"] = ref_oqs
    try:
        pkg = types.ModuleType("refcrypto2")
        pkg.__path__ = [str(REF / "crypto")]
        sys.modules["refcrypto2"] = pkg
        for name in ("algorithm_base", "key_exchange"):
            spec = importlib.util.spec_from_file_location(f"refcrypto2.{name}", REF / "crypto" / f"{name}.py")
            m = importlib.util.module_from_spec(spec)
            sys.modules[f"refcrypto2.{name}"] = m
            spec.loader.exec_module(m)
        ke = sys.modules["refcrypto2.key_exchange"]
        alg = ke.MLKEMKeyExchange(5)
        assert alg.variant == "ML-KEM-1024" and alg.name == "ML-KEM (Level 5)"
        import qrkem
        if qrkem.device_count() == 0:
            # no GPU here: the reference surface must surface the library's error, not fall back
            with pytest.raises(RuntimeError, match="Can not generate keypair"):
                alg.generate_keypair()
        else:  # pragma: no cover (GPU box has no /root/reference)
            pk, sk = alg.generate_keypair()
            ct, ss = alg.encapsulate(pk)
            assert alg.decapsulate(sk, ct) == ss
    finally:
        sys.modules.pop("oqs", None)
