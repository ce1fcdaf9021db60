"""GPU parity: the HIP path (through the C-ABI) against the CPU oracle.

Bit-exact comparisons only (integer/byte work).  Sizes are chosen so the oracle
finishes in seconds; the full BASELINE config (1 Mi x 4 KiB) is compared in
full against the multi-threaded C oracle.
"""
import hashlib
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

EDGE_LENS = [0, 1, 19, 20, 55, 56, 57, 63, 64, 65, 119, 120, 127, 128, 1024, 4050, 4096, 65536]
EDGE_N = [1, 2, 3, 4, 5, 7, 8, 9, 15, 16, 17, 255, 256, 257, 511, 512, 513, 1000, 1023, 1024,
          1025, 65535, 65536, 65537, 70001]
SEED = 0x6E616B65


def _torch():
    import torch
    assert torch.cuda.is_available(), "GPU tests need a visible device"
    return torch


def _dev(torch, arr: np.ndarray):
    return torch.from_numpy(np.ascontiguousarray(arr)).cuda()


def _bind(torch, ctx):
    ctx.set_stream(torch.cuda.current_stream().cuda_stream)


def test_leaf_hash_edge_lengths_host_api(nkv, oracle):
    _lib, ctx = nkv
    L = _lib.lib()
    lens = np.array(EDGE_LENS * 3, dtype=np.uint64)
    off = np.zeros(lens.size, np.uint64)
    off[1:] = np.cumsum(lens[:-1] + 3)  # ragged, unaligned source offsets
    data = oracle.splitmix64_bytes(int(off[-1] + lens[-1]) + 1, SEED)
    out = np.zeros((lens.size, 20), np.uint8)
    _lib.check(L.nkv_leaf_hash(ctx.h, _lib.p8(data), _lib.p64(off), _lib.p64(lens), lens.size, _lib.p8(out)))
    want = oracle.leaf_hashes(data, off, lens)
    assert np.array_equal(out, want)
    for i in range(lens.size):  # independent check against OpenSSL
        v = data[int(off[i]):int(off[i] + lens[i])].tobytes()
        assert out[i].tobytes() == hashlib.sha1(v).digest()


@pytest.mark.parametrize("shift", list(range(16)))
def test_leaf_hash_every_alignment_device(nkv, oracle, shift):
    """Unaligned in-place hashing (nkv_leaf_hash_dev): every start alignment, every tail length."""
    torch = _torch()
    _lib, ctx = nkv
    _bind(torch, ctx)
    L = _lib.lib()
    lens = np.array(EDGE_LENS + list(range(0, 200)), dtype=np.uint64)
    off = np.zeros(lens.size, np.uint64)
    off[1:] = np.cumsum(((lens[:-1] + 15) // 16) * 16 + 16)
    off += shift
    nbytes = int(off[-1] + lens[-1])
    data = oracle.splitmix64_bytes(nbytes, SEED + shift)
    d_data, d_off, d_len = _dev(torch, data), _dev(torch, off), _dev(torch, lens)
    d_nodes = torch.zeros(lens.size * 20, dtype=torch.uint8, device="cuda")
    _lib.check(L.nkv_leaf_hash_dev(ctx.h, d_data.data_ptr(), d_off.data_ptr(), d_len.data_ptr(),
                                   lens.size, d_nodes.data_ptr()))
    torch.cuda.synchronize()
    got = d_nodes.cpu().numpy().reshape(-1, 20)
    assert np.array_equal(got, oracle.leaf_hashes(data, off, lens))


@pytest.mark.parametrize("bucket", [1, 0])
def test_leaf_hash_mixed_wave_alignment(nkv, oracle, bucket):
    """Lanes of one wavefront with different alignments and lengths (with and
    without length bucketing)."""
    torch = _torch()
    _lib, ctx = nkv
    _bind(torch, ctx)
    ctx.set_option(_lib.NKV_OPT_BUCKET, bucket)
    L = _lib.lib()
    rng = np.random.default_rng(7)
    n = 5000
    lens = rng.integers(0, 3000, n).astype(np.uint64)
    off = np.zeros(n, np.uint64)
    off[1:] = np.cumsum(lens[:-1] + rng.integers(0, 17, n - 1).astype(np.uint64))
    data = oracle.splitmix64_bytes(int(off[-1] + lens[-1]), SEED)
    d_data, d_off, d_len = _dev(torch, data), _dev(torch, off), _dev(torch, lens)
    d_nodes = torch.zeros(L.nkv_total_nodes(n) * 20, dtype=torch.uint8, device="cuda")
    _lib.check(L.nkv_tree_from_values_dev(ctx.h, d_data.data_ptr(), d_off.data_ptr(), d_len.data_ptr(),
                                          n, d_nodes.data_ptr()))
    torch.cuda.synchronize()
    got = d_nodes.cpu().numpy().reshape(-1, 20)
    want = oracle.tree_from_digests(oracle.leaf_hashes(data, off, lens))
    ctx.set_option(_lib.NKV_OPT_BUCKET, 2)
    assert np.array_equal(got, want)


@pytest.mark.parametrize("load", [4, 11])
def test_mixed_sizes_log_uniform(nkv, oracle, load):
    """BASELINE configs[2] shape at reduced count: log-uniform 64 B - 64 KiB values,
    packed back to back (unaligned), every load path."""
    torch = _torch()
    _lib, ctx = nkv
    _bind(torch, ctx)
    L = _lib.lib()
    rng = np.random.default_rng(0x6E616B66)
    n = 6000
    lens = np.floor(2.0 ** rng.uniform(6, 16, n)).astype(np.uint64)
    off = np.zeros(n, np.uint64)
    off[1:] = np.cumsum(lens[:-1])
    data = oracle.splitmix64_bytes(int(lens.sum()), 0x6E616B66)
    d_data, d_off, d_len = _dev(torch, data), _dev(torch, off), _dev(torch, lens)
    d_nodes = torch.zeros(L.nkv_total_nodes(n) * 20, dtype=torch.uint8, device="cuda")
    ctx.set_option(_lib.NKV_OPT_LEAF_LOAD, load)
    try:
        _lib.check(L.nkv_tree_from_values_dev(ctx.h, d_data.data_ptr(), d_off.data_ptr(), d_len.data_ptr(),
                                              n, d_nodes.data_ptr()))
        torch.cuda.synchronize()
    finally:
        ctx.set_option(_lib.NKV_OPT_LEAF_LOAD, 4)  # the default
    want = oracle.tree_from_digests(oracle.leaf_hashes(data, off, lens, threads=8))
    assert np.array_equal(d_nodes.cpu().numpy().reshape(-1, 20), want)
    # aligned copy of the same values (host API path packs at 16 B)
    nodes = np.zeros((L.nkv_total_nodes(n), 20), np.uint8)
    _lib.check(L.nkv_tree_from_values(ctx.h, _lib.p8(data), _lib.p64(off), _lib.p64(lens), n, None,
                                      _lib.p8(nodes), None))
    assert np.array_equal(nodes, want)


@pytest.mark.parametrize("waves", [1, 2, 3])
@pytest.mark.parametrize("n,packed", [(1, True), (63, True), (65, False), (3001, True), (3001, False),
                                      (20000, True)])
def test_ragged_queue_paths(nkv, oracle, waves, n, packed):
    """Length-sorted ragged batches through the work-queue kernel (groups pulled
    from both ends, claim flags at the meeting point, the pipelined ring of
    value-relative chunks with explicit vmcnt / lgkmcnt waits) at 1-3 waves per
    SIMD.  Packed = back to back (unaligned); otherwise 16-B aligned starts."""
    torch = _torch()
    _lib, _ = nkv
    ctx = _lib.Context(0)
    _bind(torch, ctx)
    ctx.set_option(_lib.NKV_OPT_QUEUE_WAVES, waves)
    ctx.set_option(_lib.NKV_OPT_BUCKET, 1)
    L = _lib.lib()
    rng = np.random.default_rng(1000 * n + waves)
    lens = np.floor(2.0 ** rng.uniform(0, 15, n)).astype(np.uint64)
    lens[rng.integers(0, n, max(1, n // 50))] = 0
    step = lens if packed else (lens + 15) // 16 * 16
    off = np.zeros(n, np.uint64)
    off[1:] = np.cumsum(step[:-1])
    data = oracle.splitmix64_bytes(int(off[-1] + lens[-1]) + 1, SEED + n)
    d_data, d_off, d_len = _dev(torch, data), _dev(torch, off), _dev(torch, lens)
    d_nodes = torch.zeros(L.nkv_total_nodes(n) * 20, dtype=torch.uint8, device="cuda")
    try:
        for _ in range(2):  # the queue state is reset per launch
            d_nodes.zero_()
            _lib.check(L.nkv_tree_from_values_dev(ctx.h, d_data.data_ptr(), d_off.data_ptr(), d_len.data_ptr(),
                                                  n, d_nodes.data_ptr()))
            torch.cuda.synchronize()
            want = oracle.tree_from_digests(oracle.leaf_hashes(data, off, lens, threads=8))
            assert np.array_equal(d_nodes.cpu().numpy().reshape(-1, 20), want)
    finally:
        ctx.close()


@pytest.mark.parametrize("waves", [1, 3])
@pytest.mark.parametrize("split", [0, 1, 32, 100000])
@pytest.mark.parametrize("shape", ["uniform", "skewed"])
def test_queue_split_policies(nkv, oracle, split, shape, waves):
    """Work-queue kernel under every split regime: equal lengths (throughput-
    bound: every wave takes any group) and one very long value among short ones
    (the longest chain bounds the batch: short groups only to the non-priority
    waves), with splits that leave the non-priority waves nothing / everything."""
    torch = _torch()
    _lib, _ = nkv
    ctx = _lib.Context(0)
    _bind(torch, ctx)
    ctx.set_option(_lib.NKV_OPT_QUEUE_WAVES, waves)
    ctx.set_option(_lib.NKV_OPT_BUCKET, 1)  # equal lengths would take input order in auto mode
    L = _lib.lib()
    rng = np.random.default_rng(split + (7 if shape == "uniform" else 8))
    n = 9000
    if shape == "uniform":
        lens = np.full(n, 4050, np.uint64)
    else:
        lens = rng.integers(0, 2000, n).astype(np.uint64)
        lens[rng.integers(0, n, 5)] = 70000
    off = np.zeros(n, np.uint64)
    off[1:] = np.cumsum(lens[:-1] + 46)
    data = oracle.splitmix64_bytes(int(off[-1] + lens[-1]), SEED + split)
    d_data, d_off, d_len = _dev(torch, data), _dev(torch, off), _dev(torch, lens)
    d_nodes = torch.zeros(L.nkv_total_nodes(n) * 20, dtype=torch.uint8, device="cuda")
    ctx.set_option(_lib.NKV_OPT_QUEUE_SPLIT, split)
    try:
        _lib.check(L.nkv_tree_from_values_dev(ctx.h, d_data.data_ptr(), d_off.data_ptr(), d_len.data_ptr(),
                                              n, d_nodes.data_ptr()))
        torch.cuda.synchronize()
    finally:
        ctx.close()
    want = oracle.tree_from_digests(oracle.leaf_hashes(data, off, lens, threads=8))
    assert np.array_equal(d_nodes.cpu().numpy().reshape(-1, 20), want)


@pytest.mark.parametrize("n", EDGE_N)
def test_tree_build_from_digests(nkv, oracle, n):
    _lib, ctx = nkv
    L = _lib.lib()
    leaf20 = oracle.splitmix64_bytes(20 * n, SEED ^ n)
    nodes = np.zeros((L.nkv_total_nodes(n), 20), np.uint8)
    img = np.zeros(L.nkv_bfs_size(n), np.uint8)
    root = np.zeros(20, np.uint8)
    _lib.check(L.nkv_tree_build(ctx.h, _lib.p8(leaf20), n, _lib.p8(root), _lib.p8(nodes), _lib.p8(img)))
    want = oracle.tree_from_digests(leaf20.reshape(n, 20))
    assert np.array_equal(nodes, want)
    assert root.tobytes() == want[-1].tobytes()
    assert img.tobytes() == oracle.bfs_image(want, n)


@pytest.mark.parametrize("n", [131071, 262144, 262145, 524287, 1000003])
def test_tree_build_wide_levels(nkv, oracle, n):
    """Levels of >= 64 Ki nodes go through k_reduce2 (two levels per launch,
    odd counts and lone nodes at both of its levels) before the 8-level slabs."""
    _lib, ctx = nkv
    L = _lib.lib()
    leaf20 = oracle.splitmix64_bytes(20 * n, SEED ^ n)
    nodes = np.zeros((L.nkv_total_nodes(n), 20), np.uint8)
    root = np.zeros(20, np.uint8)
    _lib.check(L.nkv_tree_build(ctx.h, _lib.p8(leaf20), n, _lib.p8(root), _lib.p8(nodes), None))
    want = oracle.tree_from_digests(leaf20.reshape(n, 20))
    assert np.array_equal(nodes, want)


@pytest.mark.parametrize("n", [1, 2, 3, 255, 256, 257, 511, 513, 1000, 4097, 65537])
def test_tree_from_values_host(nkv, oracle, n):
    """Host API: leaf kernel, then the level reduce, then the image."""
    _lib, ctx = nkv
    L = _lib.lib()
    vlen = 100
    data = oracle.splitmix64_bytes(n * vlen, SEED + n)
    off = np.arange(n, dtype=np.uint64) * vlen
    lens = np.full(n, vlen, np.uint64)
    nodes = np.zeros((L.nkv_total_nodes(n), 20), np.uint8)
    img = np.zeros(L.nkv_bfs_size(n), np.uint8)
    _lib.check(L.nkv_tree_from_values(ctx.h, _lib.p8(data), _lib.p64(off), _lib.p64(lens), n, None,
                                      _lib.p8(nodes), _lib.p8(img)))
    want = oracle.tree_from_digests(oracle.leaf_hashes(data, off, lens))
    assert np.array_equal(nodes, want)
    assert img.tobytes() == oracle.bfs_image(want, n)


@pytest.mark.parametrize("base_off,stride,vlen", [(0, 4096, 4096), (0, 1024, 1024), (46, 4096, 4050),
                                                  (0, 4112, 4100), (3, 64, 61)])
def test_strided_device_path(nkv, oracle, base_off, stride, vlen):
    """The bench path (nkv_tree_from_strided_dev), aligned and SSTable-like unaligned."""
    torch = _torch()
    _lib, ctx = nkv
    _bind(torch, ctx)
    L = _lib.lib()
    n = 20000
    nbytes = base_off + stride * n
    d = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    _lib.check(L.nkv_fill_splitmix64_dev(ctx.h, d.data_ptr(), nbytes, SEED))
    d_nodes = torch.zeros(L.nkv_total_nodes(n) * 20, dtype=torch.uint8, device="cuda")
    _lib.check(L.nkv_tree_from_strided_dev(ctx.h, d.data_ptr() + base_off, stride, vlen, n, d_nodes.data_ptr()))
    torch.cuda.synchronize()
    host = oracle.splitmix64_bytes(nbytes, SEED)
    assert np.array_equal(d.cpu().numpy(), host), "device splitmix64 fill differs from the oracle's"
    got = d_nodes.cpu().numpy().reshape(-1, 20)
    want = oracle.tree_from_digests(oracle.leaf_hashes_strided(host[base_off:], stride, vlen, n, threads=8))
    assert np.array_equal(got, want)


@pytest.mark.parametrize("vlen,stride", [(0, 16), (64, 64), (128, 128), (192, 208), (4096, 4096), (8192, 8192)])
@pytest.mark.parametrize("n", [1, 1000, 4097])
def test_strided_whole_block_lengths(nkv, oracle, vlen, stride, n):
    """Lengths that are multiples of 64: the padding block is the same message in
    every lane and k_leaf<0, 4> runs its schedule on the scalar unit
    (sha1_pad_uniform); dead lanes in the last wave, and the empty value."""
    torch = _torch()
    _lib, ctx = nkv
    _bind(torch, ctx)
    L = _lib.lib()
    nbytes = stride * n
    d = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    _lib.check(L.nkv_fill_splitmix64_dev(ctx.h, d.data_ptr(), nbytes, SEED + vlen))
    d_nodes = torch.zeros(L.nkv_total_nodes(n) * 20, dtype=torch.uint8, device="cuda")
    _lib.check(L.nkv_tree_from_strided_dev(ctx.h, d.data_ptr(), stride, vlen, n, d_nodes.data_ptr()))
    torch.cuda.synchronize()
    host = oracle.splitmix64_bytes(nbytes, SEED + vlen)
    want = oracle.tree_from_digests(oracle.leaf_hashes_strided(host, stride, vlen, n, threads=8))
    assert np.array_equal(d_nodes.cpu().numpy().reshape(-1, 20), want)


@pytest.mark.parametrize("load", [4, 11])
def test_strided_every_load_path(nkv, oracle, load):
    torch = _torch()
    _lib, ctx = nkv
    _bind(torch, ctx)
    L = _lib.lib()
    n, vlen = 9000, 4096 + 48
    d = torch.empty(n * vlen, dtype=torch.uint8, device="cuda")
    _lib.check(L.nkv_fill_splitmix64_dev(ctx.h, d.data_ptr(), n * vlen, SEED))
    d_nodes = torch.zeros(L.nkv_total_nodes(n) * 20, dtype=torch.uint8, device="cuda")
    ctx.set_option(_lib.NKV_OPT_LEAF_LOAD, load)
    try:
        _lib.check(L.nkv_tree_from_strided_dev(ctx.h, d.data_ptr(), vlen, vlen, n, d_nodes.data_ptr()))
        torch.cuda.synchronize()
    finally:
        ctx.set_option(_lib.NKV_OPT_LEAF_LOAD, 4)  # the default
    host = oracle.splitmix64_bytes(n * vlen, SEED)
    want = oracle.tree_from_digests(oracle.leaf_hashes_strided(host, vlen, vlen, n, threads=8))
    assert np.array_equal(d_nodes.cpu().numpy().reshape(-1, 20), want)


def test_full_size_config2_bit_exact(nkv, oracle):
    """BASELINE config 2: 1 Mi leaves x 4 KiB, whole tree vs the C oracle."""
    torch = _torch()
    _lib, ctx = nkv
    _bind(torch, ctx)
    L = _lib.lib()
    n, vlen = 1 << 20, 4096
    d = torch.empty(n * vlen, dtype=torch.uint8, device="cuda")
    _lib.check(L.nkv_fill_splitmix64_dev(ctx.h, d.data_ptr(), n * vlen, SEED))
    d_nodes = torch.zeros(L.nkv_total_nodes(n) * 20, dtype=torch.uint8, device="cuda")
    _lib.check(L.nkv_tree_from_strided_dev(ctx.h, d.data_ptr(), vlen, vlen, n, d_nodes.data_ptr()))
    d_img = torch.zeros(L.nkv_bfs_size(n), dtype=torch.uint8, device="cuda")
    _lib.check(L.nkv_bfs_image_dev(ctx.h, d_nodes.data_ptr(), n, d_img.data_ptr()))
    torch.cuda.synchronize()
    got = d_nodes.cpu().numpy().reshape(-1, 20)
    img = d_img.cpu().numpy().tobytes()
    del d
    torch.cuda.empty_cache()
    host = oracle.splitmix64_bytes(n * vlen, SEED)
    want = oracle.tree_from_digests(oracle.leaf_hashes_strided(host, vlen, vlen, n, threads=16))
    del host
    assert np.array_equal(got, want)
    assert len(img) == oracle.bfs_size(n) == (2 * n - 1) * 21
    assert img == oracle.bfs_image(want, n)


def test_bfs_image_device_odd_sizes(nkv, oracle):
    torch = _torch()
    _lib, ctx = nkv
    _bind(torch, ctx)
    L = _lib.lib()
    for n in (1, 2, 3, 5, 1025, 300001):
        leaf20 = oracle.splitmix64_bytes(20 * n, n)
        want = oracle.tree_from_digests(leaf20.reshape(n, 20))
        d_nodes = _dev(torch, want.reshape(-1))
        d_img = torch.zeros(L.nkv_bfs_size(n), dtype=torch.uint8, device="cuda")
        _lib.check(L.nkv_bfs_image_dev(ctx.h, d_nodes.data_ptr(), n, d_img.data_ptr()))
        torch.cuda.synchronize()
        assert d_img.cpu().numpy().tobytes() == oracle.bfs_image(want, n)


def test_empty_tree_is_reference_error(nkv):
    _lib, ctx = nkv
    L = _lib.lib()
    rc = L.nkv_tree_build(ctx.h, None, 0, None, None, None)
    assert rc == _lib.NKV_ERR_EMPTY
    assert L.nkv_strerror(rc).decode() == "cannot build Merkle Tree from 0 nodes"
    z = np.zeros(1, np.uint64)
    assert L.nkv_tree_from_values(ctx.h, _lib.p8(np.zeros(1, np.uint8)), _lib.p64(z), _lib.p64(z), 0,
                                  None, None, None) == _lib.NKV_ERR_EMPTY


def test_deterministic_repeat(nkv, oracle):
    torch = _torch()
    _lib, ctx = nkv
    _bind(torch, ctx)
    L = _lib.lib()
    n = 100000
    d = torch.empty(n * 1024, dtype=torch.uint8, device="cuda")
    _lib.check(L.nkv_fill_splitmix64_dev(ctx.h, d.data_ptr(), n * 1024, 99))
    outs = []
    for _ in range(3):
        d_nodes = torch.zeros(L.nkv_total_nodes(n) * 20, dtype=torch.uint8, device="cuda")
        _lib.check(L.nkv_tree_from_strided_dev(ctx.h, d.data_ptr(), 1024, 1024, n, d_nodes.data_ptr()))
        torch.cuda.synchronize()
        outs.append(d_nodes.cpu().numpy())
    assert all(np.array_equal(outs[0], o) for o in outs[1:])


@pytest.mark.parametrize("bucket", [0, 1, 2])
@pytest.mark.parametrize("spread", [0, 3, 40])
def test_bucket_modes_narrow_and_wide(nkv, oracle, bucket, spread):
    """NKV_OPT_BUCKET 0 / 1 / 2 (auto: input order when the full-block counts lie
    within max(1, min/16), else sorted) on batches of 6000 unaligned values whose
    block counts spread 0, 3 and 40 around 63 blocks: every mode, same tree."""
    torch = _torch()
    _lib, _ = nkv
    ctx = _lib.Context(0)
    _bind(torch, ctx)
    ctx.set_option(_lib.NKV_OPT_BUCKET, bucket)
    L = _lib.lib()
    rng = np.random.default_rng(100 * bucket + spread)
    n = 6000
    lens = (4050 + 64 * rng.integers(-spread, spread + 1, n)).astype(np.uint64)
    off = np.zeros(n, np.uint64)
    off[1:] = np.cumsum(lens[:-1] + 46)
    data = oracle.splitmix64_bytes(int(off[-1] + lens[-1]), SEED + spread)
    d_data, d_off, d_len = _dev(torch, data), _dev(torch, off), _dev(torch, lens)
    d_nodes = torch.zeros(L.nkv_total_nodes(n) * 20, dtype=torch.uint8, device="cuda")
    try:
        _lib.check(L.nkv_tree_from_values_dev(ctx.h, d_data.data_ptr(), d_off.data_ptr(), d_len.data_ptr(),
                                              n, d_nodes.data_ptr()))
        torch.cuda.synchronize()
    finally:
        ctx.close()
    want = oracle.tree_from_digests(oracle.leaf_hashes(data, off, lens, threads=8))
    assert np.array_equal(d_nodes.cpu().numpy().reshape(-1, 20), want)


@pytest.mark.parametrize("side_gate", [0, 1])
def test_side_gate_alternating(nkv, oracle, side_gate):
    """NKV_OPT_SIDE_GATE: the gated plan's input-order kernel on the context's
    second stream (1) or in turn on its own stream (0).  Narrow, wide and narrow
    batches back to back on one context into one node buffer, read only after
    the last: each call's level 0 and levels are joined before the next call's
    kernels touch the buffer, so every tree is the oracle's."""
    torch = _torch()
    _lib, _ = nkv
    ctx = _lib.Context(0)
    _bind(torch, ctx)
    ctx.set_option(_lib.NKV_OPT_BUCKET, 2)
    ctx.set_option(_lib.NKV_OPT_SIDE_GATE, side_gate)
    L = _lib.lib()
    n = 5000
    cases = []
    for k, spread in enumerate((0, 40, 0, 40)):
        rng = np.random.default_rng(7 * k + spread)
        lens = (4050 + 64 * rng.integers(-spread, spread + 1, n)).astype(np.uint64)
        off = np.zeros(n, np.uint64)
        off[1:] = np.cumsum(lens[:-1] + 17)
        data = oracle.splitmix64_bytes(int(off[-1] + lens[-1]), SEED + 11 * k)
        cases.append((data, off, lens))
    d_nodes = torch.zeros(L.nkv_total_nodes(n) * 20, dtype=torch.uint8, device="cuda")
    outs = []
    try:
        for data, off, lens in cases:
            d_data, d_off, d_len = _dev(torch, data), _dev(torch, off), _dev(torch, lens)
            _lib.check(L.nkv_tree_from_values_dev(ctx.h, d_data.data_ptr(), d_off.data_ptr(), d_len.data_ptr(),
                                                  n, d_nodes.data_ptr()))
            outs.append(d_nodes.clone())  # torch's stream: ordered behind the call
        torch.cuda.synchronize()
    finally:
        ctx.close()
    for (data, off, lens), got in zip(cases, outs):
        want = oracle.tree_from_digests(oracle.leaf_hashes(data, off, lens, threads=8))
        assert np.array_equal(got.cpu().numpy().reshape(-1, 20), want)


@pytest.mark.parametrize("load", [4, 11])
@pytest.mark.parametrize("shift", [0, 1, 2, 15, 16, 17, 46, 48, 63])
@pytest.mark.parametrize("n,vlen,rec", [(1, 4050, 4096), (63, 4050, 4096), (3001, 4050, 4096), (777, 327, 400),
                                        (300, 63, 128), (257, 64, 130), (130, 1024, 1100)])
def test_line_pair_stage_uniform(nkv, oracle, load, shift, n, vlen, rec):
    """The staged paths (segment stage for a shared offset mod 64, 80-byte window stage, value-relative
    stream; LOAD 4 sends unaligned values there too): records-like values at every sub-line offset,
    through the offsets path and the strided path, dead lanes in the last wave."""
    torch = _torch()
    _lib, ctx = nkv
    _bind(torch, ctx)
    L = _lib.lib()
    nbytes = shift + rec * n + 64
    data = oracle.splitmix64_bytes(nbytes, SEED + shift)
    off = (np.arange(n, dtype=np.uint64) * rec + shift).astype(np.uint64)
    lens = np.full(n, vlen, np.uint64)
    want = oracle.tree_from_digests(oracle.leaf_hashes(data, off, lens, threads=8))
    d_data, d_off, d_len = _dev(torch, data), _dev(torch, off), _dev(torch, lens)
    d_nodes = torch.zeros(L.nkv_total_nodes(n) * 20, dtype=torch.uint8, device="cuda")
    d_nodes2 = torch.zeros_like(d_nodes)
    ctx.set_option(_lib.NKV_OPT_LEAF_LOAD, load)
    try:
        _lib.check(L.nkv_tree_from_values_dev(ctx.h, d_data.data_ptr(), d_off.data_ptr(), d_len.data_ptr(),
                                              n, d_nodes.data_ptr()))
        _lib.check(L.nkv_tree_from_strided_dev(ctx.h, d_data.data_ptr() + shift, rec, vlen, n,
                                               d_nodes2.data_ptr()))
        torch.cuda.synchronize()
    finally:
        ctx.set_option(_lib.NKV_OPT_LEAF_LOAD, 4)  # the default
    assert np.array_equal(d_nodes.cpu().numpy().reshape(-1, 20), want)
    assert np.array_equal(d_nodes2.cpu().numpy().reshape(-1, 20), want)


@pytest.mark.parametrize("load", [4, 11])
@pytest.mark.parametrize("spread", [1, 64, 3000])
def test_line_pair_stage_ragged_falls_back(nkv, oracle, load, spread):
    """Input order over values whose full-block counts differ inside a wave: those waves take
    the value-relative stream, equal-count waves the window or segment stage; every digest matches."""
    torch = _torch()
    _lib, ctx = nkv
    _bind(torch, ctx)
    L = _lib.lib()
    rng = np.random.default_rng(spread)
    n = 4500
    lens = (4000 + rng.integers(0, spread, n)).astype(np.uint64)
    lens[:640] = 4050  # the first ten waves have equal counts
    off = np.zeros(n, np.uint64)
    off[1:] = np.cumsum(lens[:-1] + 46)
    off += 46
    data = oracle.splitmix64_bytes(int(off[-1] + lens[-1]) + 64, SEED)
    want = oracle.tree_from_digests(oracle.leaf_hashes(data, off, lens, threads=8))
    d_data, d_off, d_len = _dev(torch, data), _dev(torch, off), _dev(torch, lens)
    d_nodes = torch.zeros(L.nkv_total_nodes(n) * 20, dtype=torch.uint8, device="cuda")
    ctx.set_option(_lib.NKV_OPT_LEAF_LOAD, load)
    ctx.set_option(_lib.NKV_OPT_BUCKET, 0)
    try:
        _lib.check(L.nkv_tree_from_values_dev(ctx.h, d_data.data_ptr(), d_off.data_ptr(), d_len.data_ptr(),
                                              n, d_nodes.data_ptr()))
        torch.cuda.synchronize()
    finally:
        ctx.set_option(_lib.NKV_OPT_LEAF_LOAD, 4)  # the default
        ctx.set_option(_lib.NKV_OPT_BUCKET, 2)
    assert np.array_equal(d_nodes.cpu().numpy().reshape(-1, 20), want)


@pytest.mark.parametrize("shift", [1, 3, 4, 17, 46, 60, 63])
@pytest.mark.parametrize("maxlen", [64, 130, 4050])
def test_shift_stage_uniform_offset_ragged_lengths(nkv, oracle, shift, maxlen):
    """NKV_OPT_LEAF_LOAD 11 (register stage of aligned 64-B segments, wave-uniform
    misalignment): one record size, so every value sits at the same offset mod 64,
    but the lengths differ (0 .. maxlen), so lanes of a wave stop at different
    blocks; the last value ends exactly at the end of the buffer."""
    torch = _torch()
    _lib, ctx = nkv
    _bind(torch, ctx)
    L = _lib.lib()
    rng = np.random.default_rng(shift * 1000 + maxlen)
    n, rec = 2000, 64 * ((maxlen + 63) // 64 + 1)
    off = (np.arange(n, dtype=np.uint64) * rec + shift).astype(np.uint64)
    lens = rng.integers(0, maxlen + 1, n).astype(np.uint64)
    lens[:64] = maxlen  # one wave of equal lengths
    lens[-1] = maxlen
    data = oracle.splitmix64_bytes(int(off[-1] + lens[-1]), SEED + shift)
    want = oracle.tree_from_digests(oracle.leaf_hashes(data, off, lens, threads=8))
    d_data, d_off, d_len = _dev(torch, data), _dev(torch, off), _dev(torch, lens)
    d_nodes = torch.zeros(L.nkv_total_nodes(n) * 20, dtype=torch.uint8, device="cuda")
    ctx.set_option(_lib.NKV_OPT_LEAF_LOAD, 11)
    ctx.set_option(_lib.NKV_OPT_BUCKET, 0)
    try:
        _lib.check(L.nkv_tree_from_values_dev(ctx.h, d_data.data_ptr(), d_off.data_ptr(), d_len.data_ptr(),
                                              n, d_nodes.data_ptr()))
        torch.cuda.synchronize()
    finally:
        ctx.set_option(_lib.NKV_OPT_LEAF_LOAD, 4)  # the default
        ctx.set_option(_lib.NKV_OPT_BUCKET, 2)
    assert np.array_equal(d_nodes.cpu().numpy().reshape(-1, 20), want)
