"""ctypes wrapper around oracle/liboracle.so -- TEST INFRASTRUCTURE ONLY.

The parity oracle for the batched KEM engine.  Only ``tests/``,
``__graft_entry__.smoke()`` (as the checker) and ``bench.py``'s cpu_baseline leg
import this module; the product path (``quantum-resistant-p2p_amd/qrkem``) never
does, and fails loudly when its HIP library is missing instead of falling back
here.

Parity status: Keccak/SHA3/SHAKE pinned against Python ``hashlib``; the NIST KAT
DRBG pinned against the published per-record seeds of the NIST PQC KAT files and
FIPS 197; ML-KEM and FrodoKEM arithmetic cross-checked between two independent
restatements (this C library and ``oracle/py``), but **unpinned against liboqs
itself** -- liboqs is absent from the reference tree (``.MISSING_LARGE_BLOBS:1``)
and its KAT digests are not available offline.
"""
from __future__ import annotations

import ctypes as ct
import os
import subprocess
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
LIB_PATH = HERE / "liboracle.so"

MLKEM_ALGS = ("ML-KEM-512", "ML-KEM-768", "ML-KEM-1024")
FRODO_SHAKE_ALGS = ("FrodoKEM-640-SHAKE", "FrodoKEM-976-SHAKE", "FrodoKEM-1344-SHAKE")
FRODO_AES_ALGS = ("FrodoKEM-640-AES", "FrodoKEM-976-AES", "FrodoKEM-1344-AES")
ALL_ALGS = MLKEM_ALGS + FRODO_SHAKE_ALGS + FRODO_AES_ALGS

_lib = None


def build() -> Path:
    subprocess.run(["make", "-s", "-C", str(HERE)], check=True)
    return LIB_PATH


def lib() -> ct.CDLL:
    global _lib
    if _lib is None:
        if not LIB_PATH.exists():
            build()
        L = ct.CDLL(str(LIB_PATH))
        P = ct.c_void_p
        L.orc_sizes.argtypes = [ct.c_char_p, ct.POINTER(ct.c_size_t)]
        for f in ("orc_keypair",):
            getattr(L, f).argtypes = [ct.c_char_p, P, P, P]
        L.orc_encaps.argtypes = [ct.c_char_p, P, P, P, P]
        L.orc_decaps.argtypes = [ct.c_char_p, P, P, P]
        L.orc_batch.argtypes = [ct.c_char_p, ct.c_int, ct.c_size_t, ct.c_int, P, P, P, P]
        L.orc_batch_status.argtypes = [ct.c_char_p, ct.c_int, ct.c_size_t, ct.c_int, P, P, P, P, P]
        L.orc_bench_coins.argtypes = [P, ct.c_size_t, ct.c_size_t, ct.c_uint64, ct.c_uint64]
        L.orc_bench_coins.restype = None
        L.orc_hash.argtypes = [ct.c_int, P, ct.c_size_t, P, ct.c_size_t]
        L.orc_hash.restype = None
        L.orc_kat_coins.argtypes = [ct.c_size_t, ct.c_size_t, ct.c_size_t, P, P, P]
        L.orc_kat_coins.restype = None
        L.orc_aes.argtypes = [P, ct.c_int, P, P]
        L.orc_aes.restype = None
        _lib = L
    return _lib


def sizes(alg: str) -> dict:
    out = (ct.c_size_t * 6)()
    if lib().orc_sizes(alg.encode(), out) != 0:
        raise ValueError(alg)
    keys = ("pk", "sk", "ct", "ss", "keypair_coins", "encaps_coins")
    return dict(zip(keys, [int(x) for x in out]))


def _buf(b: bytes):
    return ct.create_string_buffer(bytes(b), len(b))


def keypair(alg: str, coins: bytes) -> tuple[bytes, bytes]:
    s = sizes(alg)
    pk = ct.create_string_buffer(s["pk"])
    sk = ct.create_string_buffer(s["sk"])
    if lib().orc_keypair(alg.encode(), pk, sk, _buf(coins)) != 0:
        raise RuntimeError("oracle keypair failed")
    return pk.raw, sk.raw


def encaps(alg: str, pk: bytes, coins: bytes) -> tuple[bytes, bytes]:
    s = sizes(alg)
    c = ct.create_string_buffer(s["ct"])
    ss = ct.create_string_buffer(s["ss"])
    if lib().orc_encaps(alg.encode(), c, ss, _buf(pk), _buf(coins)) != 0:
        raise RuntimeError("oracle encaps failed")
    return c.raw, ss.raw


def decaps_rc(alg: str, sk: bytes, c: bytes) -> tuple[bytes, int]:
    """(ss, rc).  HQC: rc = -1 when the re-encryption check fails (ss still written),
    the OQS_KEM_decaps return liboqs gives; ML-KEM / FrodoKEM always return 0."""
    s = sizes(alg)
    ss = ct.create_string_buffer(s["ss"])
    rc = lib().orc_decaps(alg.encode(), ss, _buf(c), _buf(sk))
    return ss.raw, int(rc)


def decaps(alg: str, sk: bytes, c: bytes) -> bytes:
    ss, rc = decaps_rc(alg, sk, c)
    if rc != 0:
        raise RuntimeError("oracle decaps failed")
    return ss


def _ptr(a: np.ndarray):
    assert a.flags["C_CONTIGUOUS"]
    return a.ctypes.data_as(ct.c_void_p)


def batch_keypair(alg: str, coins: np.ndarray, threads: int = 0) -> tuple[np.ndarray, np.ndarray]:
    s = sizes(alg)
    n = coins.shape[0]
    pk = np.zeros((n, s["pk"]), np.uint8)
    sk = np.zeros((n, s["sk"]), np.uint8)
    rc = lib().orc_batch(alg.encode(), 0, n, threads or os.cpu_count(), _ptr(pk), _ptr(sk),
                         _ptr(np.ascontiguousarray(coins)), None)
    if rc:
        raise RuntimeError("oracle batch keypair failed")
    return pk, sk


def batch_encaps(alg: str, pk: np.ndarray, coins: np.ndarray, threads: int = 0):
    s = sizes(alg)
    n = pk.shape[0]
    c = np.zeros((n, s["ct"]), np.uint8)
    ss = np.zeros((n, s["ss"]), np.uint8)
    rc = lib().orc_batch(alg.encode(), 1, n, threads or os.cpu_count(), _ptr(c), _ptr(ss),
                         _ptr(np.ascontiguousarray(pk)), _ptr(np.ascontiguousarray(coins)))
    if rc:
        raise RuntimeError("oracle batch encaps failed")
    return c, ss


def batch_decaps(alg: str, sk: np.ndarray, c: np.ndarray, threads: int = 0, with_status: bool = False):
    """ss [n, ss]; with_status: (ss, status int32 [n]) with each record's decaps return code."""
    s = sizes(alg)
    n = sk.shape[0]
    ss = np.zeros((n, s["ss"]), np.uint8)
    st = np.zeros(n, np.int32)
    rc = lib().orc_batch_status(alg.encode(), 2, n, threads or os.cpu_count(), _ptr(ss), None,
                                _ptr(np.ascontiguousarray(c)), _ptr(np.ascontiguousarray(sk)),
                                _ptr(st) if with_status else None)
    if rc:
        raise RuntimeError("oracle batch decaps failed")
    return (ss, st) if with_status else ss


def bench_coins(n: int, length: int, seed: int, first_index: int = 0) -> np.ndarray:
    out = np.zeros((n, length), np.uint8)
    lib().orc_bench_coins(_ptr(out), n, length, seed, first_index)
    return out


def hash_(which: int, data: bytes, outlen: int) -> bytes:
    out = ct.create_string_buffer(outlen)
    lib().orc_hash(which, out, outlen, _buf(data), len(data))
    return out.raw


def kat_coins(count: int, kp: int, enc: int):
    kpo = np.zeros((count, kp), np.uint8)
    eno = np.zeros((count, enc), np.uint8)
    seeds = np.zeros((count, 48), np.uint8)
    lib().orc_kat_coins(count, kp, enc, _ptr(kpo), _ptr(eno), _ptr(seeds))
    return seeds, kpo, eno


def aes_block(key: bytes, block: bytes) -> bytes:
    out = ct.create_string_buffer(16)
    lib().orc_aes(_buf(key), 8 * len(key), _buf(block), out)
    return out.raw


# ---------------------------------------------------------------- HKDF-SHA256 / handshake
def _hk():
    L = lib()
    if not getattr(L, "_hk_bound", False):
        P, SZ = ct.c_void_p, ct.c_size_t
        L.orc_sha256.argtypes = [P, P, SZ]
        L.orc_sha256.restype = None
        L.orc_hkdf_sha256.argtypes = [P, SZ, P, SZ, P, SZ, P, SZ]
        L.orc_hkdf_batch.argtypes = [SZ, ct.c_int, P, SZ, P, SZ, P, P, SZ, P, SZ]
        L.orc_handshake_batch.argtypes = [ct.c_char_p, SZ, ct.c_int, P, P, P, P, P, SZ, SZ, P, P, P, P, P]
        L._hk_bound = True
    return L


def sha256(data: bytes) -> bytes:
    out = ct.create_string_buffer(32)
    _hk().orc_sha256(out, _buf(data), len(data))
    return out.raw


def hkdf_sha256(ikm: bytes, info: bytes, length: int, salt: bytes | None = None) -> bytes:
    out = ct.create_string_buffer(max(length, 1))
    rc = _hk().orc_hkdf_sha256(out, length, _buf(ikm), len(ikm), _buf(salt) if salt else None,
                               len(salt) if salt else 0, _buf(info), len(info))
    if rc:
        raise ValueError("bad HKDF length")
    return out.raw[:length]


def pack_infos(infos) -> tuple[np.ndarray, np.ndarray]:
    """list[bytes] -> (concatenated uint8, uint64 offsets [n+1])."""
    off = np.zeros(len(infos) + 1, np.uint64)
    off[1:] = np.cumsum([len(x) for x in infos])
    data = np.frombuffer(b"".join(infos) or b"\0", np.uint8).copy()
    return data, off


def batch_hkdf(ikm: np.ndarray, infos, length: int, salt: bytes | None = None, threads: int = 0) -> np.ndarray:
    n = ikm.shape[0]
    data, off = pack_infos(infos)
    okm = np.zeros((n, length), np.uint8)
    ikm = np.ascontiguousarray(ikm)
    rc = _hk().orc_hkdf_batch(n, threads or os.cpu_count(), _ptr(ikm), ikm.shape[1],
                              _buf(salt) if salt else None, len(salt) if salt else 0,
                              _ptr(data), _ptr(off), 0, _ptr(okm), length)
    if rc:
        raise RuntimeError("oracle batch hkdf failed")
    return okm


def batch_handshake(alg: str, coins_kp_i: np.ndarray, coins_kp_r: np.ndarray, coins_enc: np.ndarray,
                    infos, key_len: int, threads: int = 0):
    """Per handshake: KeyGen_i, KeyGen_r, Encaps(pk_i), HKDF, Decaps(sk_i, ct), HKDF
    (messaging.py:590, 809, 830, 845, 1038, 1068).  Returns pk_i, pk_r, ct, key_i, key_r."""
    s = sizes(alg)
    n = coins_kp_i.shape[0]
    data, off = pack_infos(infos)
    pk_i = np.zeros((n, s["pk"]), np.uint8)
    pk_r = np.zeros((n, s["pk"]), np.uint8)
    c = np.zeros((n, s["ct"]), np.uint8)
    key_i = np.zeros((n, key_len), np.uint8)
    key_r = np.zeros((n, key_len), np.uint8)
    args = [np.ascontiguousarray(x) for x in (coins_kp_i, coins_kp_r, coins_enc)]
    rc = _hk().orc_handshake_batch(alg.encode(), n, threads or os.cpu_count(), *[_ptr(x) for x in args],
                                   _ptr(data), _ptr(off), 0, key_len, _ptr(pk_i), _ptr(pk_r), _ptr(c),
                                   _ptr(key_i), _ptr(key_r))
    if rc:
        raise RuntimeError("oracle batch handshake failed")
    return pk_i, pk_r, c, key_i, key_r
