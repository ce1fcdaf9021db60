"""core/record byte format -- the input side of the Merkle step (host code, no hashing).

Layout written by record.Serialize (core/record/record.go:191-199), little endian:
  Crc u32 | Timestamp i64 | Status u8 | TypeInfo u8 | KeySize u64 | ValueSize u64 | Key | Value
TotalSize = 30 + KeySize + ValueSize (record.go:44-46); Crc = CRC-32/IEEE over
Key || Value (record.go:51).  The Merkle leaf of a record is SHA-1(Value) only
(core/sstable/sstable.go:62, core/lsmtree/lsmtree.go:211).
"""
from __future__ import annotations

import struct
import time
import zlib
from dataclasses import dataclass
from typing import Iterable, List, Tuple

import numpy as np

HEADER_SIZE = 30  # 4 + 8 + 1 + 1 + 8 + 8
RECORD_STATUS_DEFAULT = 0
RECORD_TOMBSTONE_REMOVED = 1
_HDR = struct.Struct("<IqBBQQ")


@dataclass
class Record:  # record.go:26-35
    Crc: int
    Timestamp: int
    Status: int
    TypeInfo: int
    KeySize: int
    ValueSize: int
    Key: bytes
    Value: bytes

    def TotalSize(self) -> int:  # record.go:44-46
        return HEADER_SIZE + self.KeySize + self.ValueSize

    def ToBytes(self) -> bytes:  # record.go:175-187
        return _HDR.pack(self.Crc, self.Timestamp, self.Status, self.TypeInfo, self.KeySize,
                         self.ValueSize) + self.Key + self.Value

    def IsDeleted(self) -> bool:  # record.go:96-98
        return (self.Status & RECORD_TOMBSTONE_REMOVED) == RECORD_TOMBSTONE_REMOVED


def New(key: bytes, val: bytes, timestamp: int = None) -> Record:  # record.go:49-60
    key, val = bytes(key), bytes(val)
    return Record(zlib.crc32(key + val) & 0xFFFFFFFF,
                  int(time.time()) if timestamp is None else int(timestamp),
                  RECORD_STATUS_DEFAULT, 0, len(key), len(val), key, val)


def parse(buf: bytes, off: int = 0) -> Tuple[Record, int]:
    """record.Deserialize (record.go:119-172) on an in-memory buffer: returns
    (record, next offset); raises ValueError on a CRC mismatch (the reference panics)."""
    crc, ts, st, ti, ks, vs = _HDR.unpack_from(buf, off)
    k0 = off + HEADER_SIZE
    key = bytes(buf[k0:k0 + ks])
    val = bytes(buf[k0 + ks:k0 + ks + vs])
    if len(key) != ks or len(val) != vs:
        raise EOFError("truncated record")
    if zlib.crc32(key + val) & 0xFFFFFFFF != crc:
        raise ValueError(f"Bad Record checksum (got {zlib.crc32(key + val)}, expected {crc})")
    return Record(crc, ts, st, ti, ks, vs, key, val), k0 + ks + vs


def data_table(records: Iterable[Record]) -> Tuple[bytes, np.ndarray]:
    """The Data-table byte stream (sstable/datatable.go) and each record's
    TotalSize (KeyContext.RecSize, record.go:38-41)."""
    parts: List[bytes] = []
    sizes: List[int] = []
    for r in records:
        b = r.ToBytes()
        parts.append(b)
        sizes.append(len(b))
    return b"".join(parts), np.asarray(sizes, dtype=np.uint64)


def value_spans(stream: bytes, rec_sizes: np.ndarray) -> Tuple[np.ndarray, np.ndarray]:
    """Host reference for the value locator: (offset, length) of each Value."""
    offs = np.zeros(len(rec_sizes), np.uint64)
    lens = np.zeros(len(rec_sizes), np.uint64)
    p = 0
    for i, rs in enumerate(rec_sizes):
        _, _, _, _, ks, vs = _HDR.unpack_from(stream, p)
        offs[i] = p + HEADER_SIZE + ks
        lens[i] = vs
        p += int(rs)
    return offs, lens


def checksums(stream, rec_sizes, ctx=None) -> Tuple[np.ndarray, int, int]:
    """Device CRC-32/IEEE of every record's Key || Value in a Data-table stream
    (nkv_record_crc; record.go:51 and :163-169).  Returns (checksums, number of
    records whose stored Crc differs, lowest such index or -1)."""
    import ctypes
    from nakevaleng_amd import _lib
    ctx = ctx or _lib.default_context()
    buf = np.frombuffer(bytes(stream), np.uint8) if not isinstance(stream, np.ndarray) else stream
    buf = np.ascontiguousarray(buf, dtype=np.uint8)
    sizes = np.ascontiguousarray(rec_sizes, dtype=np.uint64)
    n = sizes.size
    crc = np.zeros(max(n, 1), np.uint32)
    bad, first = ctypes.c_uint64(0), ctypes.c_uint64(0)
    _lib.check(_lib.lib().nkv_record_crc(ctx.h, _lib.p8(buf if buf.size else np.zeros(1, np.uint8)), buf.size,
                                         _lib.p64(sizes if n else np.zeros(1, np.uint64)), n,
                                         crc.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)),
                                         ctypes.byref(bad), ctypes.byref(first)))
    return crc[:n], int(bad.value), (-1 if first.value == 2**64 - 1 else int(first.value))


def verify(stream, rec_sizes, ctx=None) -> np.ndarray:
    """record.Deserialize's checksum check over a whole Data-table stream on the
    device: raises ValueError with the reference's message (record.go:166-167)
    for the first bad record, else returns the checksums."""
    crc, bad, first = checksums(stream, rec_sizes, ctx)
    if bad:
        off = int(np.sum(np.asarray(rec_sizes, dtype=np.uint64)[:first]))
        stored = _HDR.unpack_from(bytes(stream), off)[0]
        raise ValueError(f"Bad Record checksum (got {int(crc[first])}, expected {stored})")
    return crc
