"""GPU: the ds/merkletree-shaped Python mirror, the SSTable/compaction Merkle
steps and the records path, against the golden fixtures and the oracle."""
import hashlib
import json
import os

import numpy as np
import pytest

from tests.golden.make_golden import splitmix64_bytes

pytestmark = pytest.mark.gpu
GOLDEN = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "merkle_golden.json")))


@pytest.fixture(scope="module")
def mt(nkv):
    from nakevaleng_amd import merkletree
    return merkletree


def test_readme_example(mt):
    g = GOLDEN["readme"]
    t = mt.New([mt.MerkleNode(x.encode()) for x in g["leaves"]])
    assert t.Root.String() == g["root"]
    assert t.SerializeBytes().hex() == g["bfs_hex"]
    assert t.Validate() is True


def test_single_newleaf(mt):
    t = mt.New([mt.NewLeaf(b"x")])
    assert t.Root.String() == GOLDEN["single_x"]["root"]
    assert t.SerializeBytes().hex() == GOLDEN["single_x"]["bfs_hex"]


@pytest.mark.parametrize("case", GOLDEN["trees"], ids=lambda c: f"n{c['n']}x{c['value_bytes']}")
def test_newleaf_batch_then_new(mt, case, tmp_path):
    n, vlen = case["n"], case["value_bytes"]
    data = splitmix64_bytes(n * vlen, case["seed"])
    leaves = [mt.NewLeaf(data[i * vlen:(i + 1) * vlen]) for i in range(n)]
    t = mt.New(leaves)
    assert mt.root_of(t).hex() == case["root"]
    f = str(tmp_path / "db-1-0-metadata.db")
    t.Serialize(f)
    img = open(f, "rb").read()
    assert len(img) == case["bfs_len"] and hashlib.sha1(img).hexdigest() == case["bfs_sha1"]
    assert hashlib.sha1(b"".join(x.Data for x in leaves)).hexdigest() == case["leaf_digests_sha1"]
    # the materialized pointer tree serializes to the same bytes
    assert t.Root.String() == case["root"]
    assert hashlib.sha1(t.SerializeBytes()).hexdigest() == case["bfs_sha1"]
    assert t.Validate()


def test_leaf_data_before_new(mt, oracle):
    vals = [bytes([i]) * (i * 13) for i in range(40)]
    leaves = [mt.NewLeaf(v) for v in vals]
    assert leaves[7].Data == hashlib.sha1(vals[7]).digest()  # resolves the pending batch on the GPU
    t = mt.New(leaves)  # 20-byte leaves path (batch already sealed)
    want = oracle.tree_from_digests(np.frombuffer(b"".join(hashlib.sha1(v).digest() for v in vals), np.uint8))
    assert mt.root_of(t) == want[-1].tobytes()


def test_validate_detects_corruption(mt):
    t = mt.New([mt.NewLeaf(bytes([i]) * 100) for i in range(13)])
    assert t.Validate()
    leaf = t.Root
    while leaf.Left is not None:
        leaf = leaf.Left
    leaf.Data = bytes(20)
    assert not t.Validate()


def test_deserialize_root_only(mt, tmp_path):
    t = mt.New([mt.NewLeaf(bytes([i])) for i in range(100)])
    f = str(tmp_path / "m.db")
    t.Serialize(f)
    t2 = mt.MerkleTree()
    t2.Deserialize(f)
    assert t2.Root.Data == mt.root_of(t)
    assert t2.Root.Left is None and t2.Root.Right is None
    assert t2.Validate()


def test_serialize_keeps_stale_tail(mt, tmp_path):
    f = str(tmp_path / "m.db")
    big = mt.New([mt.NewLeaf(bytes([i])) for i in range(10)])
    small = mt.New([mt.NewLeaf(b"a")])
    big.Serialize(f)
    small.Serialize(f)
    blob = open(f, "rb").read()
    assert len(blob) == len(big.SerializeBytes())
    assert blob[:43] == small.SerializeBytes()


def test_empty_new_raises(mt):
    with pytest.raises(mt.MerkleTreeError, match="cannot build Merkle Tree from 0 nodes"):
        mt.New([])


@pytest.mark.parametrize("g", GOLDEN["generic"], ids=lambda g: f"n{g['n']}")
def test_generic_leaves(mt, g):
    raw = splitmix64_bytes(4096, g["seed"])
    datas, p = [], g["offset0"]
    for L in g["lens"]:
        datas.append(raw[p:p + L])
        p += L
    t = mt.New([mt.MerkleNode(d) for d in datas])
    assert mt.root_of(t).hex() == g["root"]
    img = t.SerializeBytes()
    assert len(img) == g["bfs_len"] and hashlib.sha1(img).hexdigest() == g["bfs_sha1"]


def _golden_stream():
    from nakevaleng_amd import record
    g = GOLDEN["records"]
    raw = splitmix64_bytes(1 << 16, g["seed"])
    recs, p = [], 0
    for i in range(g["n"]):
        ks, vs = 1 + raw[i] % 20, (raw[50 + i] * 7) % 300
        recs.append(record.New(raw[p:p + ks], raw[p + ks:p + ks + vs], timestamp=1700000000 + i))
        p += ks + vs
    return recs


def test_sstable_make_metadata(nkv, tmp_path):
    from nakevaleng_amd import sstable
    g = GOLDEN["records"]
    recs = _golden_stream()
    t = sstable.make_metadata(str(tmp_path) + "/", "nakevaleng", 1, 0, recs)
    blob = open(str(tmp_path / "nakevaleng-1-0-metadata.db"), "rb").read()
    assert hashlib.sha1(blob).hexdigest() == g["bfs_sha1"]


def test_metadata_from_records_in_place(nkv, tmp_path):
    from nakevaleng_amd import record, sstable
    g = GOLDEN["records"]
    stream, sizes = record.data_table(_golden_stream())
    root = sstable.make_metadata_from_records(str(tmp_path) + "/", "db", 2, 5, stream, sizes)
    assert root.hex() == g["root"]
    blob = open(str(tmp_path / "db-2-5-metadata.db"), "rb").read()
    assert hashlib.sha1(blob).hexdigest() == g["bfs_sha1"]


def test_records_path_large_and_bad_header(nkv, oracle):
    from nakevaleng_amd import _lib, lsmtree, record
    rng = np.random.default_rng(5)
    recs = [record.New(rng.bytes(int(rng.integers(1, 64))), rng.bytes(int(rng.integers(0, 5000))), timestamp=i)
            for i in range(3000)]
    stream, sizes = record.data_table(recs)
    off, ln = record.value_spans(stream, sizes)
    want = oracle.tree_from_digests(oracle.leaf_hashes(np.frombuffer(stream, np.uint8), off, ln))
    assert lsmtree.gpu_table_root((stream, sizes)) == want[-1].tobytes()
    bad = bytearray(stream)
    bad[22:30] = (10**12).to_bytes(8, "little")  # ValueSize of record 0 points past the stream
    with pytest.raises(_lib.NkvError):
        lsmtree.gpu_table_root((bytes(bad), sizes))


def test_device_locator_matches_host(nkv):
    import torch
    from nakevaleng_amd import record
    _lib, ctx = nkv
    L = _lib.lib()
    ctx.set_stream(torch.cuda.current_stream().cuda_stream)
    stream, sizes = record.data_table(_golden_stream())
    d_stream = torch.from_numpy(np.frombuffer(stream, np.uint8).copy()).cuda()
    d_sizes = torch.from_numpy(sizes.astype(np.uint64).view(np.int64)).cuda()
    n = len(sizes)
    d_roff = torch.empty(n, dtype=torch.int64, device="cuda")
    d_voff = torch.empty(n, dtype=torch.int64, device="cuda")
    d_vlen = torch.empty(n, dtype=torch.int64, device="cuda")
    _lib.check(L.nkv_record_offsets_dev(ctx.h, d_sizes.data_ptr(), n, d_roff.data_ptr()))
    _lib.check(L.nkv_locate_values_dev(ctx.h, d_stream.data_ptr(), len(stream), d_roff.data_ptr(), n,
                                       d_voff.data_ptr(), d_vlen.data_ptr()))
    torch.cuda.synchronize()
    off, ln = record.value_spans(stream, sizes)
    assert np.array_equal(d_voff.cpu().numpy().astype(np.uint64), off)
    assert np.array_equal(d_vlen.cpu().numpy().astype(np.uint64), ln)
    assert np.array_equal(d_roff.cpu().numpy().astype(np.uint64),
                          np.concatenate([[0], np.cumsum(sizes)[:-1]]).astype(np.uint64))


def test_tree_from_records_dev_async_and_bad_header(nkv, oracle):
    """nkv_tree_from_records_dev: the compaction form on a device-resident Data
    table, asynchronous with a device error flag, or synchronous without one."""
    import torch
    from nakevaleng_amd import record
    _lib, ctx = nkv
    L = _lib.lib()
    ctx.set_stream(torch.cuda.current_stream().cuda_stream)
    rng = np.random.default_rng(21)
    recs = [record.New(rng.bytes(int(rng.integers(1, 50))), rng.bytes(int(rng.integers(0, 9000))), timestamp=i)
            for i in range(2500)]
    stream, sizes = record.data_table(recs)
    n = len(sizes)
    roff = np.zeros(n, np.uint64)
    roff[1:] = np.cumsum(np.asarray(sizes, np.uint64)[:-1])
    off, ln = record.value_spans(stream, sizes)
    want = oracle.tree_from_digests(oracle.leaf_hashes(np.frombuffer(stream, np.uint8), off, ln))
    d_stream = torch.from_numpy(np.frombuffer(stream, np.uint8).copy()).cuda()
    d_roff = torch.from_numpy(roff.view(np.int64)).cuda()
    d_nodes = torch.zeros(L.nkv_total_nodes(n) * 20, dtype=torch.uint8, device="cuda")
    d_err = torch.full((1,), 7, dtype=torch.int32, device="cuda")
    _lib.check(L.nkv_tree_from_records_dev(ctx.h, d_stream.data_ptr(), len(stream), d_roff.data_ptr(), n,
                                           d_nodes.data_ptr(), d_err.data_ptr()))
    torch.cuda.synchronize()
    assert int(d_err.item()) == 0
    assert np.array_equal(d_nodes.cpu().numpy().reshape(-1, 20), want)
    bad = np.frombuffer(stream, np.uint8).copy()
    bad[int(roff[7]) + 22:int(roff[7]) + 30] = np.frombuffer(np.uint64(10**12).tobytes(), np.uint8)
    d_bad = torch.from_numpy(bad).cuda()
    _lib.check(L.nkv_tree_from_records_dev(ctx.h, d_bad.data_ptr(), len(stream), d_roff.data_ptr(), n,
                                           d_nodes.data_ptr(), d_err.data_ptr()))
    torch.cuda.synchronize()
    assert int(d_err.item()) == 1
    assert L.nkv_tree_from_records_dev(ctx.h, d_bad.data_ptr(), len(stream), d_roff.data_ptr(), n,
                                       d_nodes.data_ptr(), None) == _lib.NKV_ERR_INVALID
    # the grid-fold slots restore themselves: a good stream after a bad one
    # reports no error
    d_err.fill_(7)
    _lib.check(L.nkv_tree_from_records_dev(ctx.h, d_stream.data_ptr(), len(stream), d_roff.data_ptr(), n,
                                           d_nodes.data_ptr(), d_err.data_ptr()))
    torch.cuda.synchronize()
    assert int(d_err.item()) == 0
    assert np.array_equal(d_nodes.cpu().numpy().reshape(-1, 20), want)


@pytest.mark.parametrize("n", [4096, 5000, 300000])
def test_tree_from_records_dev_uniform_gated(nkv, oracle, n):
    """Uniform records (the SSTable case) through the device-range plan: k_locate
    measures the range in its grid fold, the input-order kernel runs, twice in a
    row (the fold slots must be back at their identities between calls)."""
    import torch
    _lib, ctx = nkv
    L = _lib.lib()
    ctx.set_stream(torch.cuda.current_stream().cuda_stream)
    rb, ks = 512, 16
    body = oracle.splitmix64_bytes(n * rb, n).reshape(n, rb)
    body[:, 14:22] = np.frombuffer(np.uint64(ks).tobytes(), np.uint8)
    body[:, 22:30] = np.frombuffer(np.uint64(rb - 30 - ks).tobytes(), np.uint8)
    roff = np.arange(n, dtype=np.uint64) * rb
    want = oracle.tree_from_digests(oracle.leaf_hashes(body.reshape(-1), roff + 30 + ks,
                                                       np.full(n, rb - 30 - ks, np.uint64), threads=8))
    d_stream = torch.from_numpy(body.reshape(-1).copy()).cuda()
    d_roff = torch.from_numpy(roff.view(np.int64)).cuda()
    d_err = torch.full((1,), 7, dtype=torch.int32, device="cuda")
    for _ in range(2):
        d_nodes = torch.zeros(L.nkv_total_nodes(n) * 20, dtype=torch.uint8, device="cuda")
        _lib.check(L.nkv_tree_from_records_dev(ctx.h, d_stream.data_ptr(), n * rb, d_roff.data_ptr(), n,
                                               d_nodes.data_ptr(), d_err.data_ptr()))
        torch.cuda.synchronize()
        assert int(d_err.item()) == 0
        assert np.array_equal(d_nodes.cpu().numpy().reshape(-1, 20), want)


@pytest.mark.parametrize("n", [300, 5000])
def test_record_paths_wild_offsets(nkv, n):
    """Record offsets far outside the stream (near 2^64, where offset + 30
    wraps) are reported as bad headers by every device record path, and no
    kernel reads through them."""
    import torch
    _lib, ctx = nkv
    L = _lib.lib()
    ctx.set_stream(torch.cuda.current_stream().cuda_stream)
    rb, ks = 256, 16
    n_ = n
    body = np.zeros((n_, rb), np.uint8)
    body[:, 14:22] = np.frombuffer(np.uint64(ks).tobytes(), np.uint8)
    body[:, 22:30] = np.frombuffer(np.uint64(rb - 30 - ks).tobytes(), np.uint8)
    slen = n_ * rb
    roff = np.arange(n_, dtype=np.uint64) * rb
    for i, w in ((1, 2**64 - 8), (n_ // 2, 2**64 - 29), (n_ - 2, slen - 29), (n_ - 1, slen)):
        roff[i] = w
    d_stream = torch.from_numpy(body.reshape(-1)).cuda()
    d_roff = torch.from_numpy(roff.view(np.int64)).cuda()
    d_nodes = torch.zeros(L.nkv_total_nodes(n_) * 20, dtype=torch.uint8, device="cuda")
    d_err = torch.zeros(1, dtype=torch.int32, device="cuda")
    _lib.check(L.nkv_tree_from_records_dev(ctx.h, d_stream.data_ptr(), slen, d_roff.data_ptr(), n_,
                                           d_nodes.data_ptr(), d_err.data_ptr()))
    d_stats = torch.zeros(3, dtype=torch.int64, device="cuda")
    _lib.check(L.nkv_record_crc_dev(ctx.h, d_stream.data_ptr(), slen, d_roff.data_ptr(), n_, None,
                                    d_stats.data_ptr()))
    torch.cuda.synchronize()
    assert int(d_err.item()) == 1
    assert int(d_stats[2].item()) == 1
    d_stats.zero_()
    _lib.check(L.nkv_tree_verify_records_dev(ctx.h, d_stream.data_ptr(), slen, d_roff.data_ptr(), n_,
                                             d_nodes.data_ptr(), None, d_stats.data_ptr()))
    torch.cuda.synchronize()
    assert int(d_stats[2].item()) == 1
    d_bits = torch.zeros(4 * 1024, dtype=torch.uint8, device="cuda")
    assert L.nkv_bloom_insert_records_dev(ctx.h, d_stream.data_ptr(), slen, d_roff.data_ptr(), n_, 32768, 3, 1,
                                          d_bits.data_ptr()) == _lib.NKV_ERR_INVALID
    d_voff = torch.empty(n_, dtype=torch.int64, device="cuda")
    d_vlen = torch.empty(n_, dtype=torch.int64, device="cuda")
    assert L.nkv_locate_values_dev(ctx.h, d_stream.data_ptr(), slen, d_roff.data_ptr(), n_, d_voff.data_ptr(),
                                   d_vlen.data_ptr()) == _lib.NKV_ERR_INVALID
    torch.cuda.synchronize()
