"""CPU: the C-ABI library loads, exports every symbol include/qrkem.h declares,
and answers the registry / struct queries the reference's ctypes wrapper makes
(quantum_resistant_p2p/vendor/oqs.py:192-198, 241-253, 271-280, 396-421).
No KEM compute is called here unless a GPU is present."""
import ctypes as ct
import re
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
HEADER = ROOT / "include" / "qrkem.h"


def declared_functions():
    text = HEADER.read_text()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    names = re.findall(r"\b([A-Za-z_][A-Za-z0-9_]*)\s*\(", text)
    skip = {"OQS_STATUS", "if", "sizeof", "extern", "keypair", "encaps", "decaps", "defined"}
    return sorted({n for n in names if (n.startswith("OQS_") or n.startswith("qrk_")) and n not in skip})


def test_library_exports_every_declared_symbol():
    import qrkem
    out = subprocess.run(["nm", "-D", "--defined-only", str(qrkem.LIB_PATH)], capture_output=True, text=True,
                         check=True).stdout
    exported = {line.split()[-1] for line in out.splitlines() if line.strip()}
    missing = [n for n in declared_functions() if n not in exported]
    assert not missing, missing
    assert len(declared_functions()) >= 30


class OQSKemStruct(ct.Structure):
    # the prefix layout oqs.py:241-253 maps onto OQS_KEM*
    _fields_ = [("method_name", ct.c_char_p), ("alg_version", ct.c_char_p), ("claimed_nist_level", ct.c_ubyte),
                ("ind_cca", ct.c_ubyte), ("length_public_key", ct.c_size_t), ("length_secret_key", ct.c_size_t),
                ("length_ciphertext", ct.c_size_t), ("length_shared_secret", ct.c_size_t),
                ("keypair_cb", ct.c_void_p), ("encaps_cb", ct.c_void_p), ("decaps_cb", ct.c_void_p)]


@pytest.mark.parametrize("alg,sizes,level", [
    ("ML-KEM-512", (800, 1632, 768, 32), 1),
    ("ML-KEM-768", (1184, 2400, 1088, 32), 3),
    ("ML-KEM-1024", (1568, 3168, 1568, 32), 5),
])
def test_oqs_kem_struct_prefix(alg, sizes, level):
    from qrkem._native import LIB
    p = LIB.OQS_KEM_new(alg.encode())
    assert p
    s = ct.cast(p, ct.POINTER(OQSKemStruct)).contents
    assert s.method_name.decode() == alg
    assert s.claimed_nist_level == level and s.ind_cca == 1
    assert (s.length_public_key, s.length_secret_key, s.length_ciphertext, s.length_shared_secret) == sizes
    assert s.keypair_cb and s.encaps_cb and s.decaps_cb
    LIB.OQS_KEM_free(p)


def test_registry_and_errors():
    from qrkem import oqs
    sup = oqs.get_supported_kem_mechanisms()
    en = oqs.get_enabled_kem_mechanisms()
    assert {"ML-KEM-512", "ML-KEM-768", "ML-KEM-1024"} <= set(en)
    assert set(en) <= set(sup)
    # every KEM the reference selects (key_exchange.py:75-79, 206-210, 332-343) is enabled
    assert {"HQC-128", "HQC-192", "HQC-256"} <= set(en)
    assert not any(n.startswith("Kyber") for n in sup)  # different bytes from ML-KEM
    with pytest.raises(oqs.MechanismNotSupportedError):
        oqs.KeyEncapsulation("NoSuchKEM")
    with pytest.raises(oqs.MechanismNotSupportedError):
        oqs.KeyEncapsulation("BIKE-L1")
    assert oqs.oqs_version()
    from qrkem._native import LIB
    assert not LIB.OQS_KEM_new(b"NoSuchKEM")
    assert LIB.OQS_KEM_alg_is_enabled(b"ML-KEM-768") == 1
    assert LIB.OQS_KEM_alg_is_enabled(b"HQC-256") == 1


# liboqs 0.12 sizes of the 2023-04-30 HQC (pk, sk, ct, ss) and our coin lengths
HQC_SIZES = {"HQC-128": (2249, 2305, 4433, 64, 96, 32), "HQC-192": (4522, 4586, 8978, 64, 104, 40),
             "HQC-256": (7245, 7317, 14421, 64, 112, 48)}


@pytest.mark.parametrize("alg", sorted(HQC_SIZES))
def test_hqc_sizes(alg):
    from qrkem._native import LIB
    out = (ct.c_size_t * 6)()
    assert LIB.qrk_kem_sizes(alg.encode(), out) == 0
    assert tuple(out) == HQC_SIZES[alg]
    p = LIB.OQS_KEM_new(alg.encode())
    assert p
    LIB.OQS_KEM_free(p)


def test_mem_cleanse():
    from qrkem._native import LIB
    buf = ct.create_string_buffer(b"\xaa" * 64, 64)
    LIB.OQS_MEM_cleanse(ct.addressof(buf), 64)
    assert buf.raw == bytes(64)


def test_no_cpu_fallback_without_gpu():
    """With no HIP device every KEM call fails loudly (never a CPU path)."""
    import qrkem
    if qrkem.device_count() > 0:
        pytest.skip("GPU present")
    from qrkem import oqs
    k = oqs.KeyEncapsulation("ML-KEM-768")
    with pytest.raises(RuntimeError, match="Can not generate keypair"):
        k.generate_keypair()
    assert "no HIP device" in qrkem.last_error()
    with pytest.raises(RuntimeError, match="Can not encapsulate secret"):
        k.encap_secret(bytes(1184))
    k2 = oqs.KeyEncapsulation("ML-KEM-768", bytes(2400))
    with pytest.raises(RuntimeError, match="Can not decapsulate secret"):
        k2.decap_secret(bytes(1088))
    from qrkem.batch import BatchKEM
    with pytest.raises(RuntimeError, match="cannot create a context"):
        BatchKEM("ML-KEM-768")


def test_encap_secret_length_semantics():
    """Longer-than-pk input raises ValueError (ctypes create_string_buffer, oqs.py:338-341)."""
    from qrkem import oqs
    k = oqs.KeyEncapsulation("ML-KEM-512")
    with pytest.raises(ValueError):
        k.encap_secret(bytes(801))


LEVELS = {"ML-KEM-512": 1, "ML-KEM-768": 3, "ML-KEM-1024": 5, "FrodoKEM-640-AES": 1, "FrodoKEM-640-SHAKE": 1,
          "FrodoKEM-976-AES": 3, "FrodoKEM-976-SHAKE": 3, "FrodoKEM-1344-AES": 5, "FrodoKEM-1344-SHAKE": 5,
          "HQC-128": 1, "HQC-192": 3, "HQC-256": 5}


@pytest.mark.parametrize("alg", sorted(LEVELS))
def test_details_claimed_level_from_struct(alg):
    """details / attributes come from the OQS_KEM struct, as oqs.py:273-280 reads them (HQC's
    '128' is a security-bit count, not a level: the struct says 1/3/5)."""
    from qrkem import oqs
    k = oqs.KeyEncapsulation(alg)
    assert k.claimed_nist_level == LEVELS[alg] and k.details["claimed_nist_level"] == LEVELS[alg]
    assert k.method_name.decode() == alg and k.details["name"] == alg
    s = oqs.kem_sizes(alg)
    assert (k.length_public_key, k.length_secret_key, k.length_ciphertext, k.length_shared_secret) == (
        s["length_public_key"], s["length_secret_key"], s["length_ciphertext"], s["length_shared_secret"])
    k.free()


@pytest.mark.parametrize("alg", ["ML-KEM-768", "FrodoKEM-976-SHAKE", "HQC-128"])
def test_derand_coins_length_checked(alg):
    """The library reads exactly the coin length: a wrong-length seed raises instead of being
    read past its end."""
    from qrkem import oqs
    k = oqs.KeyEncapsulation(alg)
    s = oqs.kem_sizes(alg)
    with pytest.raises(ValueError, match="keypair coins"):
        k.generate_keypair_derand(bytes(s["length_keypair_coins"] - 1))
    with pytest.raises(ValueError, match="encaps coins"):
        k.encap_secret_derand(bytes(s["length_public_key"]), bytes(s["length_encaps_coins"] + 1))
