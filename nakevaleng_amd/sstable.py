"""The Merkle step of the SSTable writer (core/sstable/sstable.go), on the MI355X.

  make_metadata              sstable.makeMetadata           sstable.go:58-74
  make_table_secondaries     Merkle part of MakeTableSecondaries   sstable.go:35-47
  make_metadata_from_records the same, hashing Values in place inside the
                             serialized Data table
  make_filter_contents       the bits of sstable.makeFilter  sstable.go:49-56 (8f row 4)
  make_filter_from_records   the same over the keys of a serialized Data table
  table_filename             util/filename.Table             filename.go:58-65, 300-309

Everything else the writer produces (Data, Index, Summary files; the Filter's
gob encoding) is outside this path and unchanged.
"""
from __future__ import annotations

from typing import Iterable, List, Optional

import numpy as np

from . import _lib
from .merkletree import MerkleNode, MerkleTree, MerkleTreeError, New, NewLeaf
from .record import Record

TYPE_METADATA = "metadata"


def table_filename(path: str, dbname: str, level: int, run: int, filetype: str = TYPE_METADATA) -> str:
    if not path.endswith("/"):
        raise ValueError("Table() :: relativePath must end with '/'")
    if level <= 0:
        raise ValueError("Level must be a positive integer!")
    if run < 0:
        raise ValueError("Run must be a non-negative integer!")
    return f"{path}{dbname}-{level}-{run}-{filetype}.db"


def make_metadata(path: str, dbname: str, level: int, run: int, records: Iterable[Record]) -> MerkleTree:
    """sstable.go:58-74: NewLeaf(rec.Value) per record, New, Serialize."""
    leaves = [NewLeaf(r.Value) for r in records]
    tree = New(leaves)  # raises MerkleTreeError("cannot build Merkle Tree from 0 nodes") like the panic
    tree.Serialize(table_filename(path, dbname, level, run))
    return tree


def make_table_secondaries(path: str, dbname: str, level: int, run: int,
                           merkleleaves: List[MerkleNode]) -> MerkleTree:
    """Merkle part of sstable.go:35-47 (leaves collected by lsmtree.merge, lsmtree.go:211)."""
    tree = New(merkleleaves)
    tree.Serialize(table_filename(path, dbname, level, run))
    return tree


def make_metadata_from_records(path: str, dbname: str, level: int, run: int, stream: bytes,
                               rec_sizes: np.ndarray, device: Optional[int] = None) -> bytes:
    """Same output file as make_metadata, straight from the Data-table bytes and
    KeyContext.RecSize list: values are located and hashed on the device
    (nkv_tree_from_records) on `device` (None: the process's device).  Returns the
    root digest."""
    n = len(rec_sizes)
    if n == 0:
        raise MerkleTreeError("cannot build Merkle Tree from 0 nodes")
    L = _lib.lib()
    ctx = _lib.default_context(device)
    buf = np.frombuffer(bytes(stream) + b"\0", dtype=np.uint8)
    rs = np.ascontiguousarray(rec_sizes, dtype=np.uint64)
    img = np.zeros(L.nkv_bfs_size(n), np.uint8)
    root = np.zeros(20, np.uint8)
    _lib.check(L.nkv_tree_from_records(ctx.h, _lib.p8(buf), buf.size - 1, _lib.p64(rs), n,
                                       _lib.p8(root), None, _lib.p8(img)), "MakeTable")
    fname = table_filename(path, dbname, level, run)
    _lib.check(L.nkv_write_file(fname.encode(), _lib.p8(img), img.size), f"Serialize({fname})")
    return root.tobytes()


def make_filter_contents(keys, seed: int, false_positive_rate: float = 0.01, ctx=None):
    """sstable.makeFilter (sstable.go:49-56) minus the gob file: bloomfilter.New(
    len(keys), 0.01), Insert(key) for every key, on the device.  Returns the
    filter (M, K, HashSeeds, Contents).  The reference's seed is the clock."""
    from . import bloomfilter
    bf = bloomfilter.New(len(keys), false_positive_rate, seed=seed, ctx=ctx)
    bf.InsertMany(keys)
    bf.Contents  # noqa: B018 -- one device batch
    return bf


def make_filter_from_records(stream, rec_sizes, seed: int, false_positive_rate: float = 0.01, ctx=None):
    """makeFilter over the keys of a serialized Data table (KeyContext.Key is the
    record's Key), hashed in place on the device (nkv_bloom_from_records)."""
    import ctypes
    from . import bloomfilter
    sizes = np.ascontiguousarray(rec_sizes, dtype=np.uint64)
    bf = bloomfilter.New(int(sizes.size), false_positive_rate, seed=seed, ctx=ctx)
    buf = np.frombuffer(bytes(stream), np.uint8) if not isinstance(stream, np.ndarray) else stream
    buf = np.ascontiguousarray(buf, dtype=np.uint8)
    bits = np.zeros((bf.M + 7) // 8, np.uint8)
    ctx = ctx or _lib.default_context()
    _lib.check(_lib.lib().nkv_bloom_from_records(ctx.h, _lib.p8(buf if buf.size else np.zeros(1, np.uint8)),
                                                 buf.size, _lib.p64(sizes if sizes.size else np.zeros(1, np.uint64)),
                                                 sizes.size, bf.M, bf.K, bf.HashSeeds[0] if bf.K else 0,
                                                 _lib.p8(bits)))
    bf._contents = bytearray(bits.tobytes())
    return bf
