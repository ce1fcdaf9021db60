"""GPU: the host-buffer API through the pipelined pinned staging (host_stage.cpp).

Tiny staging chunks (4-16 KiB) and several gather threads force every value,
record stream and output to cross chunk and thread boundaries at arbitrary
byte positions; results must equal the oracle bit for bit (digests, every tree
level, the Serialize image, checksums, filter bits)."""
import ctypes

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

STAGINGS = [(4096, 1), (4096, 4), (12288, 3), (16384, 16)]


@pytest.fixture(params=STAGINGS, ids=lambda p: f"chunk{p[0]}-t{p[1]}")
def sctx(request, nkv):
    _lib, _ = nkv
    ctx = _lib.Context(0)
    ctx.set_option(_lib.NKV_OPT_STAGE_CHUNK, request.param[0])
    ctx.set_option(_lib.NKV_OPT_HOST_THREADS, request.param[1])
    yield _lib, ctx
    ctx.close()


def _ragged(rng, n, lmax):
    ln = rng.integers(0, lmax + 1, n).astype(np.uint64)
    ln[: min(n, 5)] = [0, 1, 55, 64, 4097][: min(n, 5)]
    gap = rng.integers(0, 9, n).astype(np.uint64)
    off = np.zeros(n, np.uint64)
    off[1:] = np.cumsum(ln[:-1] + gap[:-1])
    data = rng.integers(0, 256, int(off[-1] + ln[-1]) + 1, dtype=np.uint8)
    perm = rng.permutation(n)  # values in any order in memory
    return data, off[perm].copy(), ln[perm].copy()


def test_tree_from_values_staged(sctx, oracle):
    _lib, ctx = sctx
    L = _lib.lib()
    rng = np.random.default_rng(11)
    data, off, ln = _ragged(rng, 700, 3000)
    n = ln.size
    nodes = np.zeros((L.nkv_total_nodes(n), 20), np.uint8)
    img = np.zeros(L.nkv_bfs_size(n), np.uint8)
    root = np.zeros(20, np.uint8)
    _lib.check(L.nkv_tree_from_values(ctx.h, _lib.p8(data), _lib.p64(off), _lib.p64(ln), n, _lib.p8(root),
                                      _lib.p8(nodes), _lib.p8(img)))
    want = oracle.tree_from_digests(oracle.leaf_hashes(data, off, ln))
    assert np.array_equal(nodes, want)
    assert img.tobytes() == oracle.bfs_image(want, n)
    assert root.tobytes() == want[-1].tobytes()


def test_leaf_hash_and_tree_build_staged(sctx, oracle):
    _lib, ctx = sctx
    L = _lib.lib()
    rng = np.random.default_rng(12)
    data, off, ln = _ragged(rng, 1500, 200)
    n = ln.size
    leaves = np.zeros((n, 20), np.uint8)
    _lib.check(L.nkv_leaf_hash(ctx.h, _lib.p8(data), _lib.p64(off), _lib.p64(ln), n, _lib.p8(leaves)))
    want = oracle.leaf_hashes(data, off, ln)
    assert np.array_equal(leaves, want)
    tree = oracle.tree_from_digests(want)
    nodes = np.zeros_like(tree)
    img = np.zeros(L.nkv_bfs_size(n), np.uint8)
    _lib.check(L.nkv_tree_build(ctx.h, _lib.p8(leaves), n, None, _lib.p8(nodes), _lib.p8(img)))
    assert np.array_equal(nodes, tree)
    assert img.tobytes() == oracle.bfs_image(tree, n)


def _records(rng, n):
    from nakevaleng_amd import record
    recs = [record.New(rng.bytes(int(rng.integers(1, 40))), rng.bytes(int(rng.integers(0, 2500))), timestamp=i)
            for i in range(n)]
    return record.data_table(recs)


def test_records_crc_and_filter_staged(sctx, oracle):
    from nakevaleng_amd import record
    _lib, ctx = sctx
    L = _lib.lib()
    rng = np.random.default_rng(13)
    stream, sizes = _records(rng, 900)
    buf = np.frombuffer(stream, np.uint8).copy()
    sizes = np.ascontiguousarray(sizes, np.uint64)
    n = sizes.size
    # Merkle step from the Data-table bytes
    off, ln = record.value_spans(stream, sizes)
    want = oracle.tree_from_digests(oracle.leaf_hashes(buf, off, ln))
    root = np.zeros(20, np.uint8)
    img = np.zeros(L.nkv_bfs_size(n), np.uint8)
    _lib.check(L.nkv_tree_from_records(ctx.h, _lib.p8(buf), buf.size, _lib.p64(sizes), n, _lib.p8(root), None,
                                       _lib.p8(img)))
    assert root.tobytes() == want[-1].tobytes()
    assert img.tobytes() == oracle.bfs_image(want, n)
    # record checksums (one corrupted value byte)
    roff = np.zeros(n, np.uint64)
    roff[1:] = np.cumsum(sizes[:-1])
    bad = buf.copy()
    j = int(np.argmax(ln > 0))
    bad[int(off[j])] ^= 0x40
    wcrc, _, _ = oracle.record_crcs(buf, roff)
    crc = np.zeros(n, np.uint32)
    nbad = np.zeros(1, np.uint64)
    first = np.zeros(1, np.uint64)
    c32 = crc.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32))
    _lib.check(L.nkv_record_crc(ctx.h, _lib.p8(bad), bad.size, _lib.p64(sizes), n, c32, _lib.p64(nbad),
                                _lib.p64(first)))
    exp = wcrc.copy()
    exp[j] = oracle.record_crcs(bad, roff[j:j + 1])[0][0]
    assert np.array_equal(crc, exp)
    assert int(nbad[0]) == 1 and int(first[0]) == j
    # filter over the record keys
    m, k = oracle.bloom_params(n, 0.01)
    bits = np.zeros((m + 7) // 8, np.uint8)
    _lib.check(L.nkv_bloom_from_records(ctx.h, _lib.p8(buf), buf.size, _lib.p64(sizes), n, m, k, 77,
                                        _lib.p8(bits)))
    kl = np.array([int.from_bytes(stream[int(r) + 14:int(r) + 22], "little") for r in roff], np.uint64)
    ko = roff + 30
    assert np.array_equal(bits, oracle.bloom_insert(buf, ko, kl, m, k, 77))
    bits2 = np.zeros_like(bits)
    _lib.check(L.nkv_bloom_build(ctx.h, _lib.p8(buf), _lib.p64(ko), _lib.p64(kl), n, m, k, 77, _lib.p8(bits2)))
    assert np.array_equal(bits2, bits)


def test_stage_options_validated(nkv):
    _lib, ctx = nkv
    L = _lib.lib()
    for key, val in ((_lib.NKV_OPT_STAGE_CHUNK, 1000), (_lib.NKV_OPT_STAGE_CHUNK, 4095),
                     (_lib.NKV_OPT_HOST_THREADS, -1), (_lib.NKV_OPT_HOST_THREADS, 100000)):
        assert L.nkv_ctx_set_option(ctx.h, key, val) == _lib.NKV_ERR_INVALID
