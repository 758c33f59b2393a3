"""CPU: qrkem's plugin classes reproduce the reference surface.

tests/golden/surface.json was captured from the reference's own
quantum_resistant_p2p/crypto/key_exchange.py (run over a stub `oqs`, see
tests/golden/make_surface_fixture.py).  Here the same constructors run against
qrkem with each captured registry patched in as the enabled-mechanism list.
"""
import json

import pytest


@pytest.fixture(scope="module")
def surface(golden_dir):
    return json.loads((golden_dir / "surface.json").read_text())


REGS = ["liboqs_full", "mlkem_only", "mlkem_frodo_shake"]


@pytest.mark.parametrize("reg", REGS)
def test_constructors_match_reference(surface, reg, monkeypatch):
    from qrkem import key_exchange as ke, oqs
    registry = tuple(surface[reg]["registry"])
    monkeypatch.setattr(oqs, "get_enabled_kem_mechanisms", lambda: registry)
    monkeypatch.setattr(ke._OQSBackedKEM, "_open", lambda self: setattr(self, "_batch", None))
    for case in surface[reg]["cases"]:
        cls = getattr(ke, case["cls"])
        if "error" in case:
            with pytest.raises(Exception) as ei:
                cls(**case["kwargs"])
            assert type(ei.value).__name__ == case["error"]
            assert str(ei.value) == case["message"]
            continue
        obj = cls(**case["kwargs"])
        assert obj.name == case["name"]
        assert obj.display_name == case["display_name"]
        assert obj.description == case["description"]
        assert obj.variant == case["variant"]
        assert obj.actual_variant == case["actual_variant"]
        assert obj.is_using_mock == case["is_using_mock"]
        assert obj.get_security_info() == case["security_info"]


def test_kyber_only_registry_is_refused(surface, monkeypatch):
    """The reference would fall back to Kyber names (key_exchange.py:97-99); qrkem refuses
    (different bytes from ML-KEM), raising the reference's own 'not found' ValueError."""
    from qrkem import key_exchange as ke, oqs
    registry = tuple(surface["kyber_only"]["registry"])
    monkeypatch.setattr(oqs, "get_enabled_kem_mechanisms", lambda: registry)
    with pytest.raises(ValueError, match="No ML-KEM or Kyber variant found for security level 3"):
        ke.MLKEMKeyExchange(3)


def test_abstract_methods(surface):
    from qrkem.key_exchange import KeyExchangeAlgorithm
    assert sorted(KeyExchangeAlgorithm.__abstractmethods__) == surface["_abstract_methods"]


def test_live_registry_constructs():
    from qrkem import MLKEMKeyExchange, KyberKeyExchange
    k = MLKEMKeyExchange()
    assert k.variant == "ML-KEM-768" and k.name == "ML-KEM (Level 3)"
    assert KyberKeyExchange is MLKEMKeyExchange
