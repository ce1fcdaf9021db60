"""CPU: host-side logic around the path (record format, filenames, sharding)."""
import json
import os
import struct
import zlib

import numpy as np
import pytest

from nakevaleng_amd import lsmtree, record, sstable
from tests.golden.make_golden import splitmix64_bytes

GOLDEN = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "merkle_golden.json")))


def test_record_layout_matches_reference():
    r = record.New(b"key1", b"value-bytes", timestamp=1700000000)
    b = r.ToBytes()
    assert r.TotalSize() == len(b) == 30 + 4 + 11
    crc, ts, st, ti, ks, vs = struct.unpack_from("<IqBBQQ", b)
    assert (crc, ts, st, ti, ks, vs) == (zlib.crc32(b"key1value-bytes"), 1700000000, 0, 0, 4, 11)
    assert b[30:34] == b"key1" and b[34:] == b"value-bytes"
    r2, nxt = record.parse(b)
    assert r2 == r and nxt == len(b)
    bad = bytearray(b)
    bad[-1] ^= 1
    with pytest.raises(ValueError, match="Bad Record checksum"):
        record.parse(bytes(bad))


def test_golden_record_stream_value_spans():
    g = GOLDEN["records"]
    raw = splitmix64_bytes(1 << 16, g["seed"])
    recs, p = [], 0
    for i in range(g["n"]):
        ks, vs = 1 + raw[i] % 20, (raw[50 + i] * 7) % 300
        key, val = raw[p:p + ks], raw[p + ks:p + ks + vs]
        p += ks + vs
        rr = record.New(key, val, timestamp=1700000000 + i)
        recs.append(rr)
    stream, sizes = record.data_table(recs)
    import hashlib
    assert hashlib.sha1(stream).hexdigest() == g["stream_sha1"]
    assert list(sizes) == g["rec_sizes"]
    off, ln = record.value_spans(stream, sizes)
    for r, o, n in zip(recs, off, ln):
        assert stream[int(o):int(o + n)] == r.Value


def test_table_filename():
    assert sstable.table_filename("data/", "nakevaleng", 2, 3) == "data/nakevaleng-2-3-metadata.db"
    with pytest.raises(ValueError):
        sstable.table_filename("data", "db", 1, 0)
    with pytest.raises(ValueError):
        sstable.table_filename("data/", "db", 0, 0)


def test_shard_round_robin():
    assert lsmtree.shard(4, 4, 2) == [2]
    assert lsmtree.shard(8, 4, 1) == [1, 5]
    assert sorted(sum((lsmtree.shard(10, 3, r) for r in range(3)), [])) == list(range(10))
