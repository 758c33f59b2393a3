"""Loader for libqrkem.so, the HIP (gfx950) KEM engine.

Plays the role ``quantum_resistant_p2p/vendor/__init__.py:11-57`` and
``vendor/oqs.py:122-183`` play for liboqs: find the shared library, load it with
ctypes, call ``OQS_init``.  Search order: ``$QRKEM_LIBRARY`` (a file), then the
in-tree build next to this module.  There is deliberately no fallback: if the
library is missing, importing ``qrkem`` raises ``RuntimeError`` (the product
path never routes to a CPU implementation).
"""
from __future__ import annotations

import ctypes as ct
import os
from pathlib import Path

HERE = Path(__file__).resolve().parent
DEFAULT_LIB = HERE / "libqrkem.so"


def library_path() -> Path:
    env = os.environ.get("QRKEM_LIBRARY")
    return Path(env) if env else DEFAULT_LIB


def _bind(lib: ct.CDLL) -> ct.CDLL:
    P, SZ = ct.c_void_p, ct.c_size_t
    sig = {
        "OQS_init": (None, []),
        "OQS_version": (ct.c_char_p, []),
        "OQS_KEM_alg_count": (SZ, []),
        "OQS_KEM_alg_identifier": (ct.c_char_p, [SZ]),
        "OQS_KEM_alg_is_enabled": (ct.c_int, [ct.c_char_p]),
        "OQS_KEM_new": (P, [ct.c_char_p]),
        "OQS_KEM_keypair": (ct.c_int, [P, P, P]),
        "OQS_KEM_keypair_derand": (ct.c_int, [P, P, P, P]),
        "OQS_KEM_encaps": (ct.c_int, [P, P, P, P]),
        "OQS_KEM_encaps_derand": (ct.c_int, [P, P, P, P, P]),
        "OQS_KEM_decaps": (ct.c_int, [P, P, P, P]),
        "OQS_KEM_free": (None, [P]),
        "OQS_MEM_cleanse": (None, [P, SZ]),
        "qrk_ctx_create": (ct.c_int, [ct.POINTER(P), ct.c_int]),
        "qrk_ctx_destroy": (None, [P]),
        "qrk_ctx_set_chunk": (ct.c_int, [P, SZ]),
        "qrk_ctx_set_streams": (ct.c_int, [P, ct.c_int]),
        "qrk_ctx_scratch_bytes": (SZ, [P]),
        "qrk_ctx_cleanse": (ct.c_int, [P]),
        "qrk_ctx_effective_chunk": (SZ, [P, ct.c_char_p]),
        "qrk_ctx_staging_residue": (ct.c_int, [P, ct.POINTER(ct.c_uint64)]),
        "qrk_kem_sizes": (ct.c_int, [ct.c_char_p, ct.POINTER(SZ)]),
        "qrk_kem_keypair_batch": (ct.c_int, [P, ct.c_char_p, SZ, P, P, P, P]),
        "qrk_kem_encaps_batch": (ct.c_int, [P, ct.c_char_p, SZ, P, P, P, P, P, P]),
        "qrk_kem_decaps_batch": (ct.c_int, [P, ct.c_char_p, SZ, P, P, P, P]),
        "qrk_kem_keypair_batch_host": (ct.c_int, [P, ct.c_char_p, SZ, P, P, P]),
        "qrk_kem_encaps_batch_host": (ct.c_int, [P, ct.c_char_p, SZ, P, P, P, P, P]),
        "qrk_kem_decaps_batch_host": (ct.c_int, [P, ct.c_char_p, SZ, P, P, P]),
        "qrk_kem_decaps_batch_status": (ct.c_int, [P, ct.c_char_p, SZ, P, P, P, P, P]),
        "qrk_kem_decaps_batch_status_host": (ct.c_int, [P, ct.c_char_p, SZ, P, P, P, P]),
        "qrk_bench_coins": (ct.c_int, [P, SZ, SZ, ct.c_uint64, ct.c_uint64, P, P]),
        "qrk_tamper": (ct.c_int, [P, SZ, SZ, ct.c_uint64, ct.c_int, P, P]),
        "qrk_digest_rows": (ct.c_int, [P, SZ, P, SZ, P, SZ, P, P]),
        "qrk_hqc_supports": (ct.c_int, [P, ct.c_char_p, ct.c_int, SZ, P, P, P]),
        "qrk_hkdf_sha256_batch": (ct.c_int, [P, SZ, P, SZ, P, SZ, P, P, SZ, P, SZ, P]),
        "qrk_handshake_batch": (ct.c_int, [P, ct.c_char_p, SZ, P, P, P, P, P, SZ, SZ, P, P, P, P, P, P, P]),
        "qrk_base64_encode_batch": (ct.c_int, [P, SZ, P, SZ, P, P]),
        "qrk_base64_decode_batch": (ct.c_int, [P, SZ, P, SZ, P, P, P]),
        "qrk_ctx_profile": (ct.c_int, [P, ct.c_int]),
        "qrk_ctx_profile_collect": (ct.c_int, [P]),
        "qrk_ctx_profile_get": (ct.c_int, [P, ct.c_int, ct.POINTER(ct.c_char_p), ct.POINTER(ct.c_double),
                                           ct.POINTER(ct.c_uint64)]),
        "qrk_last_error": (ct.c_char_p, []),
        "qrk_device_count": (ct.c_int, []),
    }
    for name, (res, args) in sig.items():
        fn = getattr(lib, name)  # AttributeError here = stale or foreign library
        fn.restype = res
        fn.argtypes = args
    return lib


def _load() -> ct.CDLL:
    path = library_path()
    if not path.exists():
        raise RuntimeError(
            f"qrkem: HIP library not found at {path}; build it with "
            "`python -c 'import __graft_entry__ as g; g.build()'` (no CPU fallback exists)")
    try:
        lib = ct.CDLL(str(path))
    except OSError as exc:
        raise RuntimeError(f"qrkem: could not load {path}: {exc}") from exc
    lib = _bind(lib)
    lib.OQS_init()
    return lib


LIB = _load()
LIB_PATH = library_path()


def last_error() -> str:
    msg = LIB.qrk_last_error()
    return msg.decode() if msg else ""
