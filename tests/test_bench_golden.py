"""CPU: the committed bench roots (tests/golden/bench_roots.json) reproduce.

bench.py checks every rank's root against this fixture on the GPU box
(VERDICT r03 item 1), so the fixture itself is re-derived here from the C
oracle: every configs[0]-sized root, and rank 0's configs[1] table in full
(1 Mi x 4 KiB, a few seconds on the container's cores).  The one-tree roots
are the tree over the ranks' leaves in order: checked at two ranks from the
two full tables.
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def test_small_roots(oracle):
    g = bench.golden()["small"]
    for r in range(8):
        data = oracle.splitmix64_bytes(g["leaves"] * g["value_bytes"], bench.SEED + r)
        d = oracle.leaf_hashes_strided(data, g["value_bytes"], g["value_bytes"], g["leaves"])
        assert oracle.tree_from_digests(d)[-1].tobytes().hex() == g["roots"][str(r)]


def test_full_size_roots_rank0_rank1_and_one_tree(oracle):
    g = bench.golden()
    n, vlen = g["sstable4k"]["leaves"], g["sstable4k"]["value_bytes"]
    assert (n, vlen) == (1 << 20, 4096) and g["seed"] == bench.SEED
    assert g["table_seed_step"] == bench.TABLE_SEED_STEP
    leaves = []
    for r in (0, 1):
        data = oracle.splitmix64_bytes(n * vlen, bench.SEED + r)
        leaves.append(oracle.leaf_hashes_strided(data, vlen, vlen, n, threads=os.cpu_count() or 8))
        del data
        assert oracle.tree_from_digests(leaves[-1])[-1].tobytes().hex() == g["sstable4k"]["roots"][str(r)][0]
    assert oracle.tree_from_digests(np.concatenate(leaves))[-1].tobytes().hex() == g["one_tree"]["roots"]["2"]
    # the driver's round-3 line printed rank 0's root (BENCH_r03.json)
    assert g["sstable4k"]["roots"]["0"][0] == "ab9972ce212a49b1492b71c001341efa9dad3dcf"


def test_records_and_mixed_roots_rank0(oracle):
    """The records configs' and the mixed config's committed roots (rank 0),
    re-derived as bench.build_tables lays the tables out."""
    g = bench.golden()
    r = g["records"]
    n, rb, ks = r["leaves"], r["record_bytes"], r["key_bytes"]
    stream = oracle.splitmix64_bytes(n * rb, bench.SEED)
    voff = np.arange(n, dtype=np.uint64) * rb + 30 + ks
    d = oracle.leaf_hashes(stream, voff, np.full(n, rb - 30 - ks, np.uint64), threads=os.cpu_count() or 8)
    del stream
    assert oracle.tree_from_digests(d)[-1].tobytes().hex() == r["roots"]["0"]
    m = g["mixed"]
    lens, off = bench.mixed_lengths(m["payload_bytes"], bench.SEED_MIXED)
    assert len(lens) == m["leaves"]["0"]
    data = oracle.splitmix64_bytes(int(lens.sum()), bench.SEED_MIXED)
    d = oracle.leaf_hashes(data, off, lens, threads=os.cpu_count() or 8)
    del data
    assert oracle.tree_from_digests(d)[-1].tobytes().hex() == m["roots"]["0"]


def test_stream_at_offset_matches_the_stream(oracle):
    """configs[4]'s committed roots are generated 1 Mi values at a time from the
    stream at a byte offset: the same bytes as the whole stream."""
    whole = oracle.splitmix64_bytes(1 << 20, bench.SEED + 3)
    for first in (8, 4096, 65536, (1 << 20) - 64):
        part = oracle.splitmix64_bytes((1 << 20) - first, bench.SEED + 3, first=first)
        assert np.array_equal(part, whole[first:])
    assert set(bench.golden()["config4"]["roots"]) == {str(r) for r in range(8)}
    assert bench.expected_roots("sstable4k", 8 << 20, 4096, 7, 1) == [bench.golden()["config4"]["roots"]["7"]]
