#!/usr/bin/env python3
"""Capture the reference plugin surface into tests/golden/surface.json.

Runs ONLY in the build container (needs /root/reference): loads the reference's
quantum_resistant_p2p/crypto/algorithm_base.py and key_exchange.py with a stub
`oqs` module (liboqs itself is absent, .MISSING_LARGE_BLOBS:1) and records, for
several "enabled mechanism" registries, what each constructor produces: name,
display_name, description, variant, get_security_info(), or the exception type
and message.  tests/test_surface.py replays the same registries against qrkem.
Only outputs (strings) are stored; no reference source is copied.
"""
from __future__ import annotations

import importlib.util
import json
import sys
import types
from pathlib import Path

REF = Path("/root/reference/quantum_resistant_p2p/crypto")
OUT = Path(__file__).resolve().parent / "surface.json"

REGISTRIES = {
    "liboqs_full": ["ML-KEM-512", "ML-KEM-768", "ML-KEM-1024", "Kyber512", "Kyber768", "Kyber1024",
                    "HQC-128", "HQC-192", "HQC-256", "FrodoKEM-640-AES", "FrodoKEM-640-SHAKE",
                    "FrodoKEM-976-AES", "FrodoKEM-976-SHAKE", "FrodoKEM-1344-AES", "FrodoKEM-1344-SHAKE"],
    "mlkem_only": ["ML-KEM-512", "ML-KEM-768", "ML-KEM-1024"],
    "mlkem_frodo_shake": ["ML-KEM-512", "ML-KEM-768", "ML-KEM-1024", "FrodoKEM-640-SHAKE",
                          "FrodoKEM-976-SHAKE", "FrodoKEM-1344-SHAKE"],
    "kyber_only": ["Kyber512", "Kyber768", "Kyber1024"],
}

CASES = [("MLKEMKeyExchange", {"security_level": lv}) for lv in (1, 3, 5, 2)] + \
        [("MLKEMKeyExchange", {})] + \
        [("HQCKeyExchange", {"security_level": lv}) for lv in (1, 3, 5, 4)] + \
        [("FrodoKEMKeyExchange", {"security_level": lv, "use_aes": aes}) for lv in (1, 3, 5, 0)
         for aes in (True, False)] + \
        [("FrodoKEMKeyExchange", {})]


def load(registry):
    stub = types.ModuleType("oqs")
    stub.get_enabled_kem_mechanisms = lambda: tuple(registry)

    class KeyEncapsulation:  # never exercised beyond construction
        def __init__(self, name, secret_key=None):
            self.name = name

    stub.KeyEncapsulation = KeyEncapsulation
    sys.modules["oqs"] = stub
    pkg = types.ModuleType("refcrypto")
    pkg.__path__ = [str(REF)]
    sys.modules["refcrypto"] = pkg
    mods = {}
    for name in ("algorithm_base", "key_exchange"):
        spec = importlib.util.spec_from_file_location(f"refcrypto.{name}", REF / f"{name}.py")
        m = importlib.util.module_from_spec(spec)
        sys.modules[f"refcrypto.{name}"] = m
        spec.loader.exec_module(m)
        mods[name] = m
    return mods["key_exchange"]


def main():
    out = {}
    for reg_name, reg in REGISTRIES.items():
        ke = load(reg)
        rows = []
        for cls, kw in CASES:
            row = {"cls": cls, "kwargs": kw}
            try:
                obj = getattr(ke, cls)(**kw)
                row.update({"name": obj.name, "display_name": obj.display_name, "description": obj.description,
                            "variant": obj.variant, "actual_variant": obj.actual_variant,
                            "is_using_mock": obj.is_using_mock, "security_info": obj.get_security_info()})
            except Exception as exc:  # noqa: BLE001
                row.update({"error": type(exc).__name__, "message": str(exc)})
            rows.append(row)
        out[reg_name] = {"registry": reg, "cases": rows}
    abstract = sorted(getattr(ke.KeyExchangeAlgorithm, "__abstractmethods__", ()))
    out["_abstract_methods"] = abstract
    OUT.write_text(json.dumps(out, indent=1))
    print(f"wrote {OUT}")


if __name__ == "__main__":
    main()
