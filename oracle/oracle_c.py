"""ctypes binding of oracle/liboracle.so (TEST INFRASTRUCTURE ONLY).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this.
Parity status: SHA-1 pinned by FIPS 180-4 KATs; tree layer "parity unpinned"
(see merkle_oracle.c header and DESIGN.md).
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_SO = os.path.join(_HERE, "liboracle.so")
_lib = None

u8p = ctypes.POINTER(ctypes.c_uint8)
u64p = ctypes.POINTER(ctypes.c_uint64)


_SO_OSSL = os.path.join(_HERE, "liboracle_ossl.so")
_ossl = None


def _make(so: str, srcs) -> None:
    srcs = [os.path.join(_HERE, f) for f in srcs] + [os.path.join(_HERE, "Makefile")]
    if not os.path.exists(so) or os.path.getmtime(so) < max(os.path.getmtime(s) for s in srcs):
        subprocess.check_call(["make", "-s", "-C", _HERE, os.path.basename(so)])


def build() -> str:
    _make(_SO, ("merkle_oracle.c", "record_crc_oracle.c", "bloom_oracle.c"))
    _make(_SO_OSSL, ("merkle_openssl.c",))
    return _SO


def ossl():
    """liboracle_ossl.so: the leaf hash + tree with OpenSSL's SHA-1 (libcrypto),
    the strongest CPU baseline (bench.py cpu_baseline)."""
    global _ossl
    if _ossl is None:
        build()
        L = ctypes.CDLL(_SO_OSSL)
        L.nkvo_ossl_sha1.argtypes = [u8p, ctypes.c_uint64, u8p]
        L.nkvo_ossl_leaf_hashes.argtypes = [u8p, u64p, u64p, ctypes.c_uint64, u8p, ctypes.c_int]
        L.nkvo_ossl_leaf_hashes_strided.argtypes = [u8p, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64, u8p,
                                                    ctypes.c_int]
        L.nkvo_ossl_tree_from_digests.argtypes = [u8p, ctypes.c_uint64, ctypes.c_int]
        L.nkvo_ossl_tree_from_digests.restype = ctypes.c_int
        _ossl = L
    return _ossl


def lib():
    global _lib
    if _lib is None:
        build()
        L = ctypes.CDLL(_SO)
        L.nkvo_sha1.argtypes = [u8p, ctypes.c_uint64, u8p]
        L.nkvo_splitmix64_fill.argtypes = [u8p, ctypes.c_uint64, ctypes.c_uint64]
        L.nkvo_splitmix64_fill_at.argtypes = [u8p, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64]
        L.nkvo_leaf_hashes.argtypes = [u8p, u64p, u64p, ctypes.c_uint64, u8p, ctypes.c_int]
        L.nkvo_leaf_hashes_strided.argtypes = [u8p, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64, u8p, ctypes.c_int]
        L.nkvo_num_levels.argtypes = [ctypes.c_uint64]
        L.nkvo_num_levels.restype = ctypes.c_int
        L.nkvo_total_nodes.argtypes = [ctypes.c_uint64]
        L.nkvo_total_nodes.restype = ctypes.c_uint64
        L.nkvo_tree_from_digests.argtypes = [u8p, ctypes.c_uint64]
        L.nkvo_tree_from_digests.restype = ctypes.c_int
        L.nkvo_flush_reps.argtypes = [u8p, u64p, u64p, ctypes.c_uint64, ctypes.c_int, ctypes.c_void_p, u8p]
        L.nkvo_flush_reps.restype = ctypes.c_double
        L.nkvo_tree_from_digests_mt.argtypes = [u8p, ctypes.c_uint64, ctypes.c_int]
        L.nkvo_tree_from_digests_mt.restype = ctypes.c_int
        L.nkvo_tree_generic.argtypes = [u8p, u64p, u64p, ctypes.c_uint64, u8p]
        L.nkvo_tree_generic.restype = ctypes.c_int
        L.nkvo_bfs_size.argtypes = [ctypes.c_uint64]
        L.nkvo_bfs_size.restype = ctypes.c_uint64
        L.nkvo_bfs_image.argtypes = [u8p, ctypes.c_uint64, u8p]
        L.nkvo_bfs_image.restype = ctypes.c_uint64
        L.nkvo_crc32.argtypes = [u8p, ctypes.c_uint64]
        L.nkvo_crc32.restype = ctypes.c_uint32
        L.nkvo_record_crcs.argtypes = [u8p, u64p, ctypes.c_uint64, ctypes.POINTER(ctypes.c_uint32), u8p]
        L.nkvo_record_crcs.restype = ctypes.c_uint64
        L.nkvo_crc32_s8.argtypes = [u8p, ctypes.c_uint64]
        L.nkvo_crc32_s8.restype = ctypes.c_uint32
        L.nkvo_crc32_clmul.argtypes = [u8p, ctypes.c_uint64]
        L.nkvo_crc32_clmul.restype = ctypes.c_uint32
        L.nkvo_verify_records.argtypes = [u8p, u64p, ctypes.c_uint64, u8p, ctypes.c_int, ctypes.c_void_p,
                                          ctypes.c_int]
        L.nkvo_verify_records.restype = ctypes.c_uint64
        L.nkvo_seal_records.argtypes = [u8p, u64p, ctypes.c_uint64, ctypes.c_int]
        L.nkvo_seal_records.restype = None
        L.nkvo_murmur3_32.argtypes = [u8p, ctypes.c_uint64, ctypes.c_uint32]
        L.nkvo_murmur3_32.restype = ctypes.c_uint32
        L.nkvo_bloom_params.argtypes = [ctypes.c_uint64, ctypes.c_double, ctypes.POINTER(ctypes.c_uint32),
                                        ctypes.POINTER(ctypes.c_uint32)]
        L.nkvo_bloom_insert.argtypes = [u8p, u64p, u64p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32,
                                        ctypes.c_uint32, u8p]
        L.nkvo_bloom_query.argtypes = [u8p, u64p, u64p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32,
                                       ctypes.c_uint32, u8p, u8p]
        _lib = L
    return _lib


def _p8(a: np.ndarray):
    return a.ctypes.data_as(u8p)


def _p64(a: np.ndarray):
    return a.ctypes.data_as(u64p)


def sha1(data: bytes) -> bytes:
    a = np.frombuffer(bytes(data) + b"\0", dtype=np.uint8)
    out = np.zeros(20, np.uint8)
    lib().nkvo_sha1(_p8(a), len(data), _p8(out))
    return out.tobytes()


def splitmix64_bytes(nbytes: int, seed: int, first: int = 0) -> np.ndarray:
    """Bytes [first, first + nbytes) of the splitmix64 stream (first: a multiple of 8)."""
    assert first % 8 == 0
    out = np.empty(max(nbytes, 1), np.uint8)
    if first:
        lib().nkvo_splitmix64_fill_at(_p8(out), nbytes, seed, first)
    else:
        lib().nkvo_splitmix64_fill(_p8(out), nbytes, seed)
    return out[:nbytes]


def leaf_hashes(base: np.ndarray, off: np.ndarray, ln: np.ndarray, threads: int = 1) -> np.ndarray:
    base = np.ascontiguousarray(base, np.uint8)
    if base.size == 0:
        base = np.zeros(1, np.uint8)
    off = np.ascontiguousarray(off, np.uint64)
    ln = np.ascontiguousarray(ln, np.uint64)
    n = off.size
    out = np.zeros((max(n, 1), 20), np.uint8)
    lib().nkvo_leaf_hashes(_p8(base), _p64(off), _p64(ln), n, _p8(out), threads)
    return out[:n]


def leaf_hashes_strided(base: np.ndarray, stride: int, L: int, n: int, threads: int = 1) -> np.ndarray:
    base = np.ascontiguousarray(base, np.uint8)
    out = np.zeros((max(n, 1), 20), np.uint8)
    lib().nkvo_leaf_hashes_strided(_p8(base), stride, L, n, _p8(out), threads)
    return out[:n]


def ossl_sha1(data: bytes) -> bytes:
    a = np.frombuffer(bytes(data) + b"\0", dtype=np.uint8)
    out = np.zeros(20, np.uint8)
    ossl().nkvo_ossl_sha1(_p8(a), len(data), _p8(out))
    return out.tobytes()


def ossl_leaf_hashes(base: np.ndarray, off: np.ndarray, ln: np.ndarray, threads: int = 1) -> np.ndarray:
    base = np.ascontiguousarray(base, np.uint8)
    if base.size == 0:
        base = np.zeros(1, np.uint8)
    off = np.ascontiguousarray(off, np.uint64)
    ln = np.ascontiguousarray(ln, np.uint64)
    n = off.size
    out = np.zeros((max(n, 1), 20), np.uint8)
    ossl().nkvo_ossl_leaf_hashes(_p8(base), _p64(off), _p64(ln), n, _p8(out), threads)
    return out[:n]


def ossl_leaf_hashes_strided(base: np.ndarray, stride: int, L: int, n: int, threads: int = 1) -> np.ndarray:
    base = np.ascontiguousarray(base, np.uint8)
    out = np.zeros((max(n, 1), 20), np.uint8)
    ossl().nkvo_ossl_leaf_hashes_strided(_p8(base), stride, L, n, _p8(out), threads)
    return out[:n]


def ossl_tree_from_digests(leaf20: np.ndarray, threads: int = 1) -> np.ndarray:
    """tree_from_digests with OpenSSL's SHA-1, wide levels over `threads`."""
    leaf20 = np.ascontiguousarray(leaf20, np.uint8).reshape(-1, 20)
    n = leaf20.shape[0]
    nodes = np.zeros((total_nodes(n), 20), np.uint8)
    nodes[:n] = leaf20
    if ossl().nkvo_ossl_tree_from_digests(_p8(nodes), n, threads) < 0:
        raise ValueError("cannot build Merkle Tree from 0 nodes")
    return nodes


def flush_us(base: np.ndarray, off: np.ndarray, ln: np.ndarray, reps: int, openssl: bool = False):
    """(microseconds per flush, root hex) of `reps` in-memory flushes on this
    thread (leaf hashes + tree + image, nkvo_flush_reps), with the portable
    SHA-1 or OpenSSL's."""
    base = np.ascontiguousarray(base, np.uint8)
    if base.size == 0:
        base = np.zeros(1, np.uint8)
    off = np.ascontiguousarray(off, np.uint64)
    ln = np.ascontiguousarray(ln, np.uint64)
    fn = ctypes.cast(ossl().nkvo_ossl_sha1, ctypes.c_void_p) if openssl else None
    root = np.zeros(20, np.uint8)
    s = lib().nkvo_flush_reps(_p8(base), _p64(off), _p64(ln), off.size, reps, fn, _p8(root))
    return s / reps * 1e6, root.tobytes().hex()


def num_levels(n: int) -> int:
    return lib().nkvo_num_levels(n)


def total_nodes(n: int) -> int:
    return lib().nkvo_total_nodes(n)


def tree_from_digests(leaf20: np.ndarray, threads: int = 1) -> np.ndarray:
    """All levels, level-major bottom-up, shape (total_nodes, 20).  Root is the last row.
    threads > 1: wide levels split over that many threads (same bytes)."""
    leaf20 = np.ascontiguousarray(leaf20, np.uint8).reshape(-1, 20)
    n = leaf20.shape[0]
    nodes = np.zeros((total_nodes(n), 20), np.uint8)
    nodes[:n] = leaf20
    rc = (lib().nkvo_tree_from_digests_mt(_p8(nodes), n, threads) if threads > 1
          else lib().nkvo_tree_from_digests(_p8(nodes), n))
    if rc < 0:
        raise ValueError("cannot build Merkle Tree from 0 nodes")
    return nodes


def tree_generic(data: np.ndarray, off: np.ndarray, ln: np.ndarray) -> np.ndarray:
    """Levels 1..top for leaves of arbitrary Data; shape (total_nodes(n) - n, 20)."""
    data = np.ascontiguousarray(data, np.uint8)
    if data.size == 0:
        data = np.zeros(1, np.uint8)
    off = np.ascontiguousarray(off, np.uint64)
    ln = np.ascontiguousarray(ln, np.uint64)
    n = off.size
    up = np.zeros((max(total_nodes(n) - n, 1), 20), np.uint8)
    if lib().nkvo_tree_generic(_p8(data), _p64(off), _p64(ln), n, _p8(up)) < 0:
        raise ValueError("cannot build Merkle Tree from 0 nodes")
    return up


def bfs_size(n: int) -> int:
    return lib().nkvo_bfs_size(n)


def bfs_image(nodes: np.ndarray, n: int) -> bytes:
    nodes = np.ascontiguousarray(nodes, np.uint8)
    img = np.zeros(max(bfs_size(n), 1), np.uint8)
    w = lib().nkvo_bfs_image(_p8(nodes), n, _p8(img))
    return img[:w].tobytes()


def crc32(data) -> int:
    """CRC-32 (IEEE) as Go's crc32.ChecksumIEEE (record.go:51)."""
    a = np.frombuffer(bytes(data), np.uint8) if not isinstance(data, np.ndarray) else data
    a = np.ascontiguousarray(a, dtype=np.uint8)
    buf = a if a.size else np.zeros(1, np.uint8)
    return int(lib().nkvo_crc32(_p8(buf), a.size))


def record_crcs(stream: np.ndarray, rec_off: np.ndarray):
    """(crc per record over key ++ value, ok flags, number of mismatches)."""
    off = np.ascontiguousarray(rec_off, dtype=np.uint64)
    n = off.size
    crc = np.zeros(max(n, 1), np.uint32)
    ok = np.zeros(max(n, 1), np.uint8)
    bad = lib().nkvo_record_crcs(_p8(stream), _p64(off if n else np.zeros(1, np.uint64)), n,
                                 crc.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)), _p8(ok))
    return crc[:n], ok[:n].astype(bool), int(bad)


def crc32_fast(data, clmul: bool) -> int:
    """The baseline's CRC-32 forms (slicing-by-8, or PCLMULQDQ folding), which
    tests/test_oracle.py pins against crc32() and zlib."""
    a = np.frombuffer(bytes(data), np.uint8) if not isinstance(data, np.ndarray) else data
    a = np.ascontiguousarray(a, dtype=np.uint8)
    buf = a if a.size else np.zeros(1, np.uint8)
    fn = lib().nkvo_crc32_clmul if clmul else lib().nkvo_crc32_s8
    return int(fn(_p8(buf), a.size))


def verify_records(stream: np.ndarray, rec_off: np.ndarray, threads: int = 1, openssl: bool = False):
    """The compaction read on the host (bench.py cpu_baseline of records_verify):
    every record's Crc over Key ++ Value checked and its Value's leaf digest.
    openssl: OpenSSL's SHA-1 and the PCLMULQDQ CRC, else the portable SHA-1 and
    slicing-by-8.  Returns (n x 20 digests, number of failed Crcs)."""
    stream = np.ascontiguousarray(stream, np.uint8)
    off = np.ascontiguousarray(rec_off, np.uint64)
    n = off.size
    out = np.zeros((max(n, 1), 20), np.uint8)
    fn = ctypes.cast(ossl().nkvo_ossl_sha1, ctypes.c_void_p) if openssl else None
    bad = lib().nkvo_verify_records(_p8(stream), _p64(off if n else np.zeros(1, np.uint64)), n, _p8(out),
                                    threads, fn, 1 if openssl else 0)
    return out[:n], int(bad)


def seal_records(stream: np.ndarray, rec_off: np.ndarray, threads: int = 1) -> None:
    """Write each record's Crc (Key ++ Value, record.go:51) into `stream` in place."""
    off = np.ascontiguousarray(rec_off, np.uint64)
    assert stream.flags.c_contiguous and stream.dtype == np.uint8
    if off.size:
        lib().nkvo_seal_records(_p8(stream), _p64(off), off.size, threads)


def murmur3_32(data, seed: int) -> int:
    """MurmurHash3_x86_32 as spaolacci/murmur3 Sum32 (bloomfilter.go:79-81)."""
    a = np.frombuffer(bytes(data), np.uint8) if not isinstance(data, np.ndarray) else data
    a = np.ascontiguousarray(a, dtype=np.uint8)
    buf = a if a.size else np.zeros(1, np.uint8)
    return int(lib().nkvo_murmur3_32(_p8(buf), a.size, seed & 0xFFFFFFFF))


def bloom_params(n: int, p: float):
    m, k = ctypes.c_uint32(0), ctypes.c_uint32(0)
    lib().nkvo_bloom_params(n, p, ctypes.byref(m), ctypes.byref(k))
    return m.value, k.value


def bloom_insert(base: np.ndarray, off: np.ndarray, ln: np.ndarray, m: int, k: int, seed0: int) -> np.ndarray:
    bits = np.zeros((m + 7) // 8, np.uint8)
    off = np.ascontiguousarray(off, dtype=np.uint64)
    ln = np.ascontiguousarray(ln, dtype=np.uint64)
    buf = base if base.size else np.zeros(1, np.uint8)
    lib().nkvo_bloom_insert(_p8(buf), _p64(off), _p64(ln), off.size, m, k, seed0 & 0xFFFFFFFF, _p8(bits))
    return bits


def bloom_query(base: np.ndarray, off: np.ndarray, ln: np.ndarray, m: int, k: int, seed0: int,
                bits: np.ndarray) -> np.ndarray:
    off = np.ascontiguousarray(off, dtype=np.uint64)
    ln = np.ascontiguousarray(ln, dtype=np.uint64)
    out = np.zeros(max(off.size, 1), np.uint8)
    buf = base if base.size else np.zeros(1, np.uint8)
    lib().nkvo_bloom_query(_p8(buf), _p64(off), _p64(ln), off.size, m, k, seed0 & 0xFFFFFFFF,
                           _p8(np.ascontiguousarray(bits)), _p8(out))
    return out[:off.size].astype(bool)
