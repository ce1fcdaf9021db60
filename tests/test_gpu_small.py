"""GPU: the one-launch small-tree path (k_small_tree, NKV_OPT_SMALL_PATH) against
the oracle, bit-exact: nodes, root and the Serialize image.

The reference engine flushes 10-record memtables and compacts 4 such runs by
default (engine/coreconf/coreconf.go:33-34, :39), so its own Merkle step is a
tree of 10..40 leaves; VERDICT r04 item 4.  The path follows NewLeaf
(ds/merkletree/merklenode.go:27-34), build (merkletree.go:31-64: the lone node
of an odd level hashed alone, at least one level above the leaves) and
Serialize (merkletree.go:67-92, merklenode.go:37-63).
"""
import ctypes
import os
import subprocess

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# lengths at every padding boundary: 0, one byte, 55/56 (one vs two padding
# blocks), 63/64/65, two blocks, ...
EDGE = [0, 1, 2, 3, 4, 15, 16, 17, 55, 56, 57, 63, 64, 65, 119, 120, 127, 128, 129, 191, 192, 200, 255, 256, 1000,
        1024, 1025, 4096]


def _values(n, seed, maxlen=None):
    rng = np.random.default_rng(seed)
    ln = np.array([EDGE[(i * 7 + seed) % len(EDGE)] for i in range(n)], np.uint64)
    if maxlen is not None:
        ln = np.minimum(ln, maxlen).astype(np.uint64)
    off = np.zeros(n, np.uint64)
    off[1:] = np.cumsum(ln[:-1])
    base = np.frombuffer(rng.bytes(int(ln.sum()) + 1), np.uint8).copy()
    return base, off, ln


def _want(oracle, base, off, ln):
    nodes = oracle.tree_from_digests(oracle.leaf_hashes(base, off, ln))
    return nodes, oracle.bfs_image(nodes, len(off))


def _run(_lib, ctx, base, off, ln):
    L = _lib.lib()
    n = len(off)
    root = np.zeros(20, np.uint8)
    nodes = np.zeros((L.nkv_total_nodes(n), 20), np.uint8)
    img = np.zeros(L.nkv_bfs_size(n), np.uint8)
    _lib.check(L.nkv_tree_from_values(ctx.h, _lib.p8(base), _lib.p64(off), _lib.p64(ln), n, _lib.p8(root),
                                      _lib.p8(nodes), _lib.p8(img)))
    return root, nodes, img.tobytes(), ctx.last_path()


@pytest.fixture
def small_ctx(nkv):
    _lib, ctx = nkv
    yield _lib, ctx
    ctx.set_option(_lib.NKV_OPT_SMALL_PATH, 1)
    ctx.set_option(_lib.NKV_OPT_SMALL_MAX_N, 1024)
    ctx.set_option(_lib.NKV_OPT_SMALL_MAX_BYTES, 1 << 20)


@pytest.mark.parametrize("mode", [1, 2, 3])
def test_small_path_every_n_1_to_1024(small_ctx, oracle, mode):
    """Every tree size n = 1..1024 (each odd level, each power of two and its
    neighbours), values at the padding-boundary lengths, bit-exact; the call
    takes the one-launch path (nkv_ctx_last_path)."""
    _lib, ctx = small_ctx
    ctx.set_option(_lib.NKV_OPT_SMALL_PATH, mode)
    for n in range(1, 1025):
        base, off, ln = _values(n, n, maxlen=256 if n > 300 else None)
        nodes_w, img_w = _want(oracle, base, off, ln)
        root, nodes, img, path = _run(_lib, ctx, base, off, ln)
        assert path == _lib.NKV_PATH_SMALL, n
        assert np.array_equal(nodes, nodes_w), n
        assert root.tobytes() == nodes_w[-1].tobytes(), n
        assert img == img_w, n


@pytest.mark.parametrize("mode", [1, 2, 3])
def test_small_path_edge_lengths_and_alignment(small_ctx, oracle, mode):
    """Every edge length at every source alignment 0..15 (the path packs values
    16-byte aligned: the source alignment must not matter)."""
    _lib, ctx = small_ctx
    ctx.set_option(_lib.NKV_OPT_SMALL_PATH, mode)
    rng = np.random.default_rng(7)
    for shift in range(16):
        ln = np.array(EDGE, np.uint64)
        off = np.zeros(len(ln), np.uint64)
        off[1:] = np.cumsum(ln[:-1])
        off += shift
        base = np.frombuffer(rng.bytes(int(ln.sum()) + shift + 1), np.uint8).copy()
        nodes_w, img_w = _want(oracle, base, off, ln)
        root, nodes, img, path = _run(_lib, ctx, base, off, ln)
        assert path == _lib.NKV_PATH_SMALL
        assert np.array_equal(nodes, nodes_w) and img == img_w, shift


def test_small_path_matches_grid_path_and_bounds(small_ctx, oracle):
    """The same batches through the grid path (NKV_OPT_SMALL_PATH 0) give the same
    bytes; batches above NKV_OPT_SMALL_MAX_N / _BYTES take the grid path."""
    _lib, ctx = small_ctx
    for n in (1, 2, 3, 10, 40, 257, 1000, 1024):
        base, off, ln = _values(n, 1000 + n)
        out = {}
        for mode in (0, 1, 2, 3):
            ctx.set_option(_lib.NKV_OPT_SMALL_PATH, mode)
            root, nodes, img, path = _run(_lib, ctx, base, off, ln)
            assert path == (_lib.NKV_PATH_GRID if mode == 0 else _lib.NKV_PATH_SMALL)
            out[mode] = (root.tobytes(), nodes.tobytes(), img)
        assert out[0] == out[1] == out[2] == out[3], n
    ctx.set_option(_lib.NKV_OPT_SMALL_PATH, 1)
    base, off, ln = _values(1025, 3, maxlen=64)
    nodes_w, img_w = _want(oracle, base, off, ln)
    root, nodes, img, path = _run(_lib, ctx, base, off, ln)
    assert path == _lib.NKV_PATH_GRID and np.array_equal(nodes, nodes_w) and img == img_w
    ctx.set_option(_lib.NKV_OPT_SMALL_MAX_N, 16)
    base, off, ln = _values(17, 4)
    assert _run(_lib, ctx, base, off, ln)[3] == _lib.NKV_PATH_GRID
    base, off, ln = _values(16, 4)
    assert _run(_lib, ctx, base, off, ln)[3] == _lib.NKV_PATH_SMALL
    ctx.set_option(_lib.NKV_OPT_SMALL_MAX_N, 1024)
    ctx.set_option(_lib.NKV_OPT_SMALL_MAX_BYTES, 4096)
    ln = np.array([4096, 1], np.uint64)
    off = np.array([0, 4096], np.uint64)
    base = np.frombuffer(np.random.default_rng(5).bytes(4098), np.uint8).copy()
    root, nodes, img, path = _run(_lib, ctx, base, off, ln)
    nodes_w, img_w = _want(oracle, base, off, ln)
    assert path == _lib.NKV_PATH_GRID and np.array_equal(nodes, nodes_w) and img == img_w
    for key, bad in ((_lib.NKV_OPT_SMALL_PATH, 4), (_lib.NKV_OPT_SMALL_PATH, -1), (_lib.NKV_OPT_SMALL_MAX_N, 1025),
                     (_lib.NKV_OPT_SMALL_MAX_BYTES, (1 << 30) + 1)):
        assert _lib.lib().nkv_ctx_set_option(ctx.h, key, bad) == _lib.NKV_ERR_INVALID


def _records(n, seed, key_lo=0, key_hi=40, val_hi=300):
    """A serialized Data table (record.go:191-199): Crc, Timestamp, Tombstone,
    TypeInfo, KeySize, ValueSize (little endian) @0..30, Key, Value."""
    rng = np.random.default_rng(seed)
    parts, sizes = [], []
    for i in range(n):
        ks = int(rng.integers(key_lo, key_hi + 1))
        vs = EDGE[(i + seed) % len(EDGE)] if i % 3 else int(rng.integers(0, val_hi + 1))
        hdr = bytearray(rng.bytes(30))
        hdr[14:22] = ks.to_bytes(8, "little")
        hdr[22:30] = vs.to_bytes(8, "little")
        rec = bytes(hdr) + rng.bytes(ks) + rng.bytes(vs)
        parts.append(rec)
        sizes.append(len(rec))
    return np.frombuffer(b"".join(parts), np.uint8).copy(), np.array(sizes, np.uint64)


@pytest.mark.parametrize("n", [1, 2, 3, 10, 40, 41, 255, 1024])
def test_small_path_records(small_ctx, oracle, n):
    """nkv_tree_from_records of a small Data table (a default-size compaction's
    output table: lsmtree.go:211 leaves = the records' Values) takes the one
    launch and matches the oracle; a header pointing outside the stream is
    refused as on the grid path."""
    _lib, ctx = small_ctx
    L = _lib.lib()
    stream, sizes = _records(n, n)
    roff = np.zeros(n, np.uint64)
    roff[1:] = np.cumsum(sizes[:-1])
    ks = np.array([int.from_bytes(stream[int(r) + 14:int(r) + 22].tobytes(), "little") for r in roff], np.uint64)
    vs = np.array([int.from_bytes(stream[int(r) + 22:int(r) + 30].tobytes(), "little") for r in roff], np.uint64)
    nodes_w, img_w = _want(oracle, stream, roff + 30 + ks, vs)
    for mode in (1, 0):
        ctx.set_option(_lib.NKV_OPT_SMALL_PATH, mode)
        root = np.zeros(20, np.uint8)
        nodes = np.zeros((L.nkv_total_nodes(n), 20), np.uint8)
        img = np.zeros(L.nkv_bfs_size(n), np.uint8)
        _lib.check(L.nkv_tree_from_records(ctx.h, _lib.p8(stream), stream.size, _lib.p64(sizes), n, _lib.p8(root),
                                           _lib.p8(nodes), _lib.p8(img)))
        assert ctx.last_path() == (_lib.NKV_PATH_SMALL if mode else _lib.NKV_PATH_GRID)
        assert np.array_equal(nodes, nodes_w) and img.tobytes() == img_w
        # the last record's ValueSize past the stream end
        bad = stream.copy()
        r = int(roff[-1])
        bad[r + 22:r + 30] = np.frombuffer((stream.size).to_bytes(8, "little"), np.uint8)
        assert L.nkv_tree_from_records(ctx.h, _lib.p8(bad), bad.size, _lib.p64(sizes), n, _lib.p8(root), None,
                                       None) == _lib.NKV_ERR_INVALID


def test_small_path_alternates_with_grid_calls(small_ctx, oracle):
    """Small and grid calls interleaved on one context (the ticket word and the
    pinned buffers are reused; a grid call between two small ones changes
    nothing)."""
    _lib, ctx = small_ctx
    for i in range(30):
        n = [5, 3000, 700, 1, 2048, 1024][i % 6]
        base, off, ln = _values(n, 50 + i, maxlen=512)
        nodes_w, img_w = _want(oracle, base, off, ln)
        root, nodes, img, path = _run(_lib, ctx, base, off, ln)
        assert path == (_lib.NKV_PATH_SMALL if n <= 1024 else _lib.NKV_PATH_GRID)
        assert np.array_equal(nodes, nodes_w) and img == img_w, (i, n)


def test_small_flush_tool_roots(oracle, tmp_path):
    """tools/small_flush.cpp (the C++ Go-API mirror at the default sizes, bench.py
    --config small_flush) in every mode: its roots equal the oracle's on the
    same generated values, and the mirror's image equals the C-ABI call's."""
    import sys
    sys.path.insert(0, ROOT)
    import bench
    from nakevaleng_amd import build as nb
    exe = nb.build_small_flush()
    shapes = [s for s in bench.SMALL_SHAPES if s[0] in ("flush_default", "compaction_default", "config0")]
    spec = [f"{n}:{lo}:{hi}:{bench.SMALL_SEED:x}" for _, n, lo, hi in shapes]
    for mode in (1, 2, 0):
        p = subprocess.run([exe, str(mode), "5", str(tmp_path)] + spec, capture_output=True, text=True, timeout=120)
        assert p.returncode == 0, p.stderr[-2000:]
        lines = [__import__("json").loads(x) for x in p.stdout.splitlines() if x.startswith("{")]
        assert len(lines) == len(shapes)
        for (name, n, lo, hi), line in zip(shapes, lines):
            data, off, ln = bench.small_shape_values(n, lo, hi)
            want = oracle.tree_from_digests(oracle.leaf_hashes(data, off, ln))[-1].tobytes().hex()
            assert line["root"] == want, (mode, name)
            assert line["path"] == (0 if mode == 0 else 1), (mode, name)


@pytest.mark.parametrize("coherent", [1, 0])
def test_small_path_reads_the_arena_in_place(small_ctx, oracle, coherent):
    """Values inside an nkv_host_alloc block (the mirrors' NewLeaf arena) at
    16-byte aligned places: with a host-coherent block (NKV_OPT_ARENA_COHERENT
    1, the default) the one-launch kernel reads them where they lie, unless
    they fit 16 KiB on a large-BAR GPU (then they are packed into device
    memory); with a default pinned block, or any unaligned place, they are
    packed first.  Every way bit-exact, and a block rewritten between calls is
    read afresh."""
    _lib, ctx = small_ctx
    L = _lib.lib()
    ctx.set_option(_lib.NKV_OPT_ARENA_COHERENT, coherent)
    cap = 1 << 20
    p = ctypes.c_void_p()
    _lib.check(L.nkv_host_alloc(ctx.h, cap, ctypes.byref(p)))
    try:
        arena = np.ctypeslib.as_array((ctypes.c_uint8 * cap).from_address(p.value))
        for rnd, (n, pad) in enumerate([(10, 16), (40, 16), (300, 16), (1024, 16), (77, 1), (10, 16), (10, 16)]):
            rng = np.random.default_rng(rnd)
            ln = np.array([EDGE[(i + rnd) % len(EDGE)] for i in range(n)], np.uint64)
            ln = np.minimum(ln, 600).astype(np.uint64)
            off = np.zeros(n, np.uint64)
            pos = 16 * rnd  # the batch does not start at the block's first byte
            for i in range(n):
                off[i] = pos
                pos += int(ln[i])
                pos = (pos + pad - 1) // pad * pad
            arena[:pos] = np.frombuffer(rng.bytes(pos), np.uint8)  # rewritten every round
            nodes_w, img_w = _want(oracle, arena[:pos].copy(), off, ln)
            root = np.zeros(20, np.uint8)
            nodes = np.zeros((L.nkv_total_nodes(n), 20), np.uint8)
            img = np.zeros(L.nkv_bfs_size(n), np.uint8)
            _lib.check(L.nkv_tree_from_values(ctx.h, ctypes.cast(p, _lib._u8p), _lib.p64(off), _lib.p64(ln), n,
                                              _lib.p8(root), _lib.p8(nodes), _lib.p8(img)))
            assert ctx.last_path() == _lib.NKV_PATH_SMALL
            assert np.array_equal(nodes, nodes_w) and img.tobytes() == img_w, (coherent, rnd)
    finally:
        _lib.check(L.nkv_host_free(ctx.h, p))
        ctx.set_option(_lib.NKV_OPT_ARENA_COHERENT, 1)


@pytest.mark.parametrize("mailbox", [0, 1])
def test_resident_service_across_idle_exits_and_contexts(nkv, oracle, mailbox):
    """NKV_OPT_SMALL_PATH 3 (the resident service): requests right after each
    other, after the service has left on its idle timeout (20 ms) and been
    started again, on a second context at the same time, and a context
    destroyed while its service waits -- every tree bit-exact, with the
    requests in device memory the host stores to (NKV_OPT_SERVICE_MAILBOX 0, a
    large-BAR GPU) and in host memory (1)."""
    import time
    _lib, _ = nkv
    ctxs = [_lib.Context(0), _lib.Context(0)]
    try:
        for c in ctxs:
            c.set_option(_lib.NKV_OPT_SMALL_PATH, 3)
            c.set_option(_lib.NKV_OPT_SERVICE_MAILBOX, mailbox)
        for k in range(60):
            n = 1 + (k * 37) % 300
            base, off, ln = _values(n, 5000 + k, maxlen=300)
            nodes_w, img_w = _want(oracle, base, off, ln)
            root, nodes, img, path = _run(_lib, ctxs[k % 2], base, off, ln)
            assert path == _lib.NKV_PATH_SMALL
            assert np.array_equal(nodes, nodes_w) and img == img_w, k
            if k % 10 == 9:
                time.sleep(0.05)  # past the idle timeout: the next call relaunches
        for c in ctxs:
            st = c.small_service_state()
            assert st["launches"] >= 2 and st["done"] == st["doorbell"]
            if mailbox == 1:
                assert st["mailbox_dev"] == 0
    finally:
        t0 = time.perf_counter()
        for c in ctxs:
            c.close()
        assert time.perf_counter() - t0 < 5.0


@pytest.mark.parametrize("mailbox", [0, 1])
@pytest.mark.parametrize("in_arena", [False, True])
def test_resident_service_inline_bound(small_ctx, oracle, in_arena, mailbox):
    """The service takes a request whose descriptors and values fit its own
    16 KiB input buffer (16 n + the 16-byte aligned value bytes <= 16384) with
    the request line, and any other one from the staging buffer -- or, for
    values at aligned places in a coherent arena block, where they lie.  Shapes
    on both sides of that bound and of the service's 256-value bound, plain
    host values and arena values: every tree bit-exact."""
    _lib, ctx = small_ctx
    L = _lib.lib()
    ctx.set_option(_lib.NKV_OPT_SMALL_PATH, 3)
    ctx.set_option(_lib.NKV_OPT_SERVICE_MAILBOX, mailbox)
    cap = 1 << 20
    p = ctypes.c_void_p()
    if in_arena:
        _lib.check(L.nkv_host_alloc(ctx.h, cap, ctypes.byref(p)))
    try:
        # (n, value length): 16 n + n * align16(len) just at, just over, well over 16 KiB
        shapes = [(256, 48), (256, 47), (255, 48), (256, 49), (10, 1615), (10, 1616), (10, 1617), (10, 1632),
                  (1, 16368), (1, 16369), (40, 4096), (257, 16), (1, 0), (256, 0)]
        for k, (n, each) in enumerate(shapes):
            rng = np.random.default_rng(900 + k)
            ln = np.full(n, each, np.uint64)
            off = np.zeros(n, np.uint64)
            off[1:] = np.cumsum((ln[:-1] + 15) // 16 * 16)  # 16-byte aligned places
            total = int(off[-1] + ln[-1]) + 1
            if in_arena:
                assert total <= cap
                buf = np.ctypeslib.as_array((ctypes.c_uint8 * cap).from_address(p.value))
                buf[:total] = np.frombuffer(rng.bytes(total), np.uint8)
                base_ptr = ctypes.cast(p, _lib._u8p)
                base = buf[:total].copy()
            else:
                base = np.frombuffer(rng.bytes(total), np.uint8).copy()
                base_ptr = _lib.p8(base)
            nodes_w, img_w = _want(oracle, base, off, ln)
            root = np.zeros(20, np.uint8)
            nodes = np.zeros((L.nkv_total_nodes(n), 20), np.uint8)
            img = np.zeros(L.nkv_bfs_size(n), np.uint8)
            _lib.check(L.nkv_tree_from_values(ctx.h, base_ptr, _lib.p64(off), _lib.p64(ln), n, _lib.p8(root),
                                              _lib.p8(nodes), _lib.p8(img)))
            assert ctx.last_path() == _lib.NKV_PATH_SMALL
            assert np.array_equal(nodes, nodes_w) and img.tobytes() == img_w, (in_arena, n, each)
    finally:
        if in_arena:
            _lib.check(L.nkv_host_free(ctx.h, p))
        ctx.set_option(_lib.NKV_OPT_SERVICE_MAILBOX, 0)


def test_resident_service_mailbox_switch(small_ctx, oracle):
    """NKV_OPT_SERVICE_MAILBOX changed while the service runs: the running
    service is stopped, the next call starts it in the other form, and every
    tree stays bit-exact; out-of-range values are refused."""
    _lib, ctx = small_ctx
    L = _lib.lib()
    ctx.set_option(_lib.NKV_OPT_SMALL_PATH, 3)
    for bad in (-1, 2):
        assert L.nkv_ctx_set_option(ctx.h, _lib.NKV_OPT_SERVICE_MAILBOX, bad) == _lib.NKV_ERR_INVALID
    forms = []
    for k, mailbox in enumerate([0, 1, 1, 0, 1, 0, 0]):
        ctx.set_option(_lib.NKV_OPT_SERVICE_MAILBOX, mailbox)
        for j in range(3):
            base, off, ln = _values(5 + 11 * k + j, 6000 + 10 * k + j, maxlen=300)
            nodes_w, img_w = _want(oracle, base, off, ln)
            root, nodes, img, path = _run(_lib, ctx, base, off, ln)
            assert path == _lib.NKV_PATH_SMALL
            assert np.array_equal(nodes, nodes_w) and img == img_w, (k, j)
        st = ctx.small_service_state()
        assert st["live"] == 1 and st["done"] == st["doorbell"]
        forms.append((mailbox, st["mailbox_dev"]))
    assert all(dev == 0 for mb, dev in forms if mb == 1)
    # a large-BAR GPU takes the device form whenever it is asked for
    assert len({dev for mb, dev in forms if mb == 0}) == 1
    ctx.set_option(_lib.NKV_OPT_SERVICE_MAILBOX, 0)


@pytest.mark.parametrize("mode", [1, 2, 3])
def test_small_path_without_image(small_ctx, oracle, mode):
    """A call that asks for no image (the mirrors' New: img_out NULL) gets the
    same nodes and root, for shapes across the service's bound (256) and the
    one-launch kernel's workgroup boundaries."""
    _lib, ctx = small_ctx
    ctx.set_option(_lib.NKV_OPT_SMALL_PATH, mode)
    L = _lib.lib()
    for n in (1, 2, 10, 40, 255, 256, 257, 513, 1024):
        base, off, ln = _values(n, 77 + n, maxlen=300)
        nodes_w, _ = _want(oracle, base, off, ln)
        nodes = np.zeros((L.nkv_total_nodes(n), 20), np.uint8)
        root = np.zeros(20, np.uint8)
        _lib.check(L.nkv_tree_from_values(ctx.h, _lib.p8(base), _lib.p64(off), _lib.p64(ln), n, _lib.p8(root),
                                          _lib.p8(nodes), None))
        assert ctx.last_path() == _lib.NKV_PATH_SMALL
        assert np.array_equal(nodes, nodes_w) and root.tobytes() == nodes_w[-1].tobytes(), n
        root2 = np.zeros(20, np.uint8)
        _lib.check(L.nkv_tree_from_values(ctx.h, _lib.p8(base), _lib.p64(off), _lib.p64(ln), n, _lib.p8(root2),
                                          None, None))
        assert root2.tobytes() == nodes_w[-1].tobytes(), n


@pytest.mark.parametrize("mode", [1, 3])
def test_small_path_host_input_form(small_ctx, oracle, mode):
    """NKV_OPT_SERVICE_MAILBOX 1: the one-launch kernel and the service take
    their packed input from host memory instead of BAR-mapped device memory;
    back to 0 in the same context, the device form again -- every n = 1..80 and
    a few larger, bit-exact in both forms, calls alternating between them."""
    _lib, ctx = small_ctx
    ctx.set_option(_lib.NKV_OPT_SMALL_PATH, mode)
    try:
        for n in list(range(1, 81)) + [255, 256, 300]:
            base, off, ln = _values(n, 9000 + n, maxlen=300)
            nodes_w, img_w = _want(oracle, base, off, ln)
            for mailbox in (1, 0):
                ctx.set_option(_lib.NKV_OPT_SERVICE_MAILBOX, mailbox)
                root, nodes, img, path = _run(_lib, ctx, base, off, ln)
                assert path == _lib.NKV_PATH_SMALL
                assert np.array_equal(nodes, nodes_w) and img == img_w, (mode, mailbox, n)
    finally:
        ctx.set_option(_lib.NKV_OPT_SERVICE_MAILBOX, 0)
