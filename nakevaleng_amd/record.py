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
