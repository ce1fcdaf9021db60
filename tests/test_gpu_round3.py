"""GPU: the round-3 C-ABI entries against the oracle.

- nkv_trees_dev: several tables per call spread over streams (compaction's runs,
  core/lsmtree/lsmtree.go:71-128; each table's tree as MakeTableSecondaries builds
  it, core/sstable/sstable.go:35-47).
- nkv_group_*: one process over several GPUs.  On the one-GPU box
  the RCCL transport runs at g = 1 (ncclCommInitAll over one device); the split
  and the table distribution run at g = 2..4 with device 0 listed repeatedly
  (copy transport): the same host logic, sub-root gather and top reduce.
- The deferred-NewLeaf arena (nkv_host_alloc / nkv_host_stream): values copied
  straight from the pinned block, the prefix streamed ahead of the call
  (sstable.go:58-74, merklenode.go:27-34).
- Stream hand-over: calls queued on one stream, the next on another.
- The clock probe behind bench.py's sclk_mhz.
Every digest is compared bit-exact with oracle/merkle_oracle.c.
"""
import ctypes
import struct
import zlib

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def dev(a):
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


def ragged(n, seed, maxlen=300):
    rng = np.random.default_rng(seed)
    ln = rng.integers(0, maxlen, n).astype(np.uint64)
    off = np.zeros(n, np.uint64)
    off[1:] = np.cumsum(ln)[:-1]
    base = np.frombuffer(rng.bytes(int(ln.sum()) + 1), np.uint8).copy()
    return base, off, ln


def records(n, vlen, seed, klen=16):
    """A Data table of n records (record.go:191-199) with correct Crcs: (stream, rec_off, val_off, vlen)."""
    rng = np.random.default_rng(seed)
    rs = 30 + klen + vlen
    buf = np.frombuffer(rng.bytes(n * rs), np.uint8).copy().reshape(n, rs)
    for i in range(n):
        kv = buf[i, 30:].tobytes()
        buf[i, 0:30] = np.frombuffer(struct.pack("<IqBBQQ", zlib.crc32(kv) & 0xFFFFFFFF, 1700000000 + i, 0, 0,
                                                 klen, vlen), np.uint8)
    rec_off = np.arange(n, dtype=np.uint64) * rs
    return buf.reshape(-1), rec_off, rec_off + 30 + klen, np.full(n, vlen, np.uint64)


def want_tree(oracle, base, off, ln):
    return oracle.tree_from_digests(oracle.leaf_hashes(base, off, ln, threads=8))


def nodes_buf(L, n):
    return torch.empty(L.nkv_total_nodes(n) * 20, dtype=torch.uint8, device="cuda")


def host_nodes(t):
    return t.cpu().numpy().reshape(-1, 20)


def make_tables(_lib, L, oracle):
    """Five tables of every kind: (nkv_table, expected nodes, keep-alive tensors)."""
    out = []
    # STRIDED: 5000 x 1000 B
    data = np.frombuffer(np.random.default_rng(1).bytes(5000 * 1000), np.uint8).copy()
    d = dev(data)
    nb = nodes_buf(L, 5000)
    out.append((_lib.table(_lib.NKV_TABLE_STRIDED, nb.data_ptr(), 5000, base=d.data_ptr(), stride=1000, length=1000),
                oracle.tree_from_digests(oracle.leaf_hashes_strided(data, 1000, 1000, 5000)), nb, [d]))
    # VALUES: ragged, unaligned
    base, off, ln = ragged(3001, 2)
    db, do, dl = dev(base), dev(off.view(np.int64)), dev(ln.view(np.int64))
    nb = nodes_buf(L, 3001)
    out.append((_lib.table(_lib.NKV_TABLE_VALUES, nb.data_ptr(), 3001, base=db.data_ptr(), off=do.data_ptr(),
                           lens=dl.data_ptr()), want_tree(oracle, base, off, ln), nb, [db, do, dl]))
    # RECORDS: 4100 records of 1000-B values (the auto plan: >= 4096 values)
    s, ro, vo, vl = records(4100, 1000, 3)
    ds, dr = dev(s), dev(ro.view(np.int64))
    err = torch.full((1,), 7, dtype=torch.int32, device="cuda")
    nb = nodes_buf(L, 4100)
    out.append((_lib.table(_lib.NKV_TABLE_RECORDS, nb.data_ptr(), 4100, base=ds.data_ptr(), base_len=s.size,
                           off=dr.data_ptr(), err=err.data_ptr()), want_tree(oracle, s, vo, vl), nb, [ds, dr, err]))
    # VERIFY: 700 records, every Crc right
    s, ro, vo, vl = records(700, 333, 4, klen=5)
    ds, dr = dev(s), dev(ro.view(np.int64))
    stats = torch.zeros(3, dtype=torch.int64, device="cuda")
    crc = torch.zeros(700, dtype=torch.int32, device="cuda")
    nb = nodes_buf(L, 700)
    out.append((_lib.table(_lib.NKV_TABLE_VERIFY, nb.data_ptr(), 700, base=ds.data_ptr(), base_len=s.size,
                           off=dr.data_ptr(), crc=crc.data_ptr(), stats=stats.data_ptr()),
                want_tree(oracle, s, vo, vl), nb, [ds, dr, stats, crc]))
    # STRIDED with one leaf (the >= 1 level rule)
    data1 = np.frombuffer(b"x" * 64, np.uint8).copy()
    d1 = dev(data1)
    nb = nodes_buf(L, 1)
    out.append((_lib.table(_lib.NKV_TABLE_STRIDED, nb.data_ptr(), 1, base=d1.data_ptr(), stride=64, length=64),
                oracle.tree_from_digests(oracle.leaf_hashes_strided(data1, 64, 64, 1)), nb, [d1]))
    return out


@pytest.mark.parametrize("lanes", [1, 2, 3])
def test_trees_dev_every_kind(nkv, oracle, lanes):
    _lib, ctx = nkv
    L = _lib.lib()
    tabs = make_tables(_lib, L, oracle)
    ctx.set_stream(torch.cuda.current_stream().cuda_stream)
    ctx.set_option(_lib.NKV_OPT_TABLE_LANES, lanes)
    try:
        for _ in range(2):  # twice: lanes reused, pass flags alternate
            for t in tabs:
                t[2].zero_()
            ctx.trees([t[0] for t in tabs])
            torch.cuda.synchronize()
            for t, want, nb, keep in tabs:
                assert np.array_equal(host_nodes(nb), want), t.kind
        assert int(tabs[2][3][2].item()) == 0  # RECORDS err word written
        assert tabs[3][3][2].cpu().tolist() == [0, -1, 0]  # VERIFY: no bad Crc
    finally:
        ctx.set_option(_lib.NKV_OPT_TABLE_LANES, 2)


def test_trees_dev_bad_table_then_recovers(nkv, oracle):
    """A table the call refuses (unknown kind, empty table) among good ones
    returns an error with every lane joined; the context's next call is right."""
    _lib, ctx = nkv
    L = _lib.lib()
    tabs = make_tables(_lib, L, oracle)
    ctx.set_option(_lib.NKV_OPT_TABLE_LANES, 3)
    try:
        for bad in (_lib.table(99, tabs[0][2].data_ptr(), 5), _lib.table(_lib.NKV_TABLE_STRIDED, 0, 0)):
            with pytest.raises(_lib.NkvError):
                ctx.trees([tabs[0][0], bad, tabs[1][0]])
            ctx.sync()
        for t in tabs:
            t[2].zero_()
        ctx.trees([t[0] for t in tabs])
        ctx.sync()
        for t, want, nb, keep in tabs:
            assert np.array_equal(host_nodes(nb), want), t.kind
    finally:
        ctx.set_option(_lib.NKV_OPT_TABLE_LANES, 2)


def test_trees_dev_records_err_null(nkv, oracle):
    """RECORDS tables without an err word: the call reports a header outside the
    stream as NKV_ERR_INVALID (after a sync), as nkv_tree_from_records_dev does."""
    _lib, ctx = nkv
    L = _lib.lib()
    s, ro, vo, vl = records(300, 100, 5)
    ds = dev(s)
    good, bad = dev(ro.view(np.int64)), ro.copy()
    bad[17] = s.size - 10  # header runs past the stream's end
    dbad = dev(bad.view(np.int64))
    n1, n2 = nodes_buf(L, 300), nodes_buf(L, 300)
    t_ok = _lib.table(_lib.NKV_TABLE_RECORDS, n1.data_ptr(), 300, base=ds.data_ptr(), base_len=s.size,
                      off=good.data_ptr())
    t_bad = _lib.table(_lib.NKV_TABLE_RECORDS, n2.data_ptr(), 300, base=ds.data_ptr(), base_len=s.size,
                       off=dbad.data_ptr())
    ctx.trees([t_ok, t_ok])
    ctx.sync()
    assert np.array_equal(host_nodes(n1), want_tree(oracle, s, vo, vl))
    with pytest.raises(_lib.NkvError):
        ctx.trees([t_ok, t_bad])


def test_group_rccl_one_gpu(nkv, oracle):
    """g = 1 over RCCL: ncclCommInitAll, the roots all-gather, four tables
    (configs[3]'s lsm_run_max = 4 runs, reduced record count) and one split tree."""
    _lib, _ = nkv
    L = _lib.lib()
    with _lib.Group([0]) as grp:
        assert grp.size == 1 and grp.transport == _lib.NKV_TRANSPORT_RCCL
        # four tables of 4 KiB records' values, one after another on member 0
        n, vlen = 8192, 4096 - 46
        keep, tabs, wants = [], [], []
        for t in range(4):
            s, ro, vo, vl = records(n, vlen, 10 + t)
            ds, dr = dev(s), dev(ro.view(np.int64))
            err = torch.zeros(1, dtype=torch.int32, device="cuda")
            nb = nodes_buf(L, n)
            keep += [ds, dr, err, nb]
            tabs.append(_lib.table(_lib.NKV_TABLE_RECORDS, nb.data_ptr(), n, base=ds.data_ptr(), base_len=s.size,
                                   off=dr.data_ptr(), err=err.data_ptr()))
            wants.append(want_tree(oracle, s, vo, vl)[-1].tobytes())
        roots = np.zeros(4 * 20, np.uint8)
        arr = (_lib.NkvTable * 4)(*tabs)
        _lib.check(L.nkv_group_trees_dev(grp.h, arr, 4, _lib.p8(roots)))
        assert [roots[20 * t:20 * t + 20].tobytes() for t in range(4)] == wants
        # the bare all-gather of one root
        r = keep[3][-20:]
        src = (ctypes.c_void_p * 1)(r.data_ptr())
        got = np.zeros(20, np.uint8)
        _lib.check(L.nkv_group_roots_allgather(grp.h, src, None, _lib.p8(got)))
        assert got.tobytes() == wants[0]
        # a root in host memory is refused before RCCL sees it
        bad = (ctypes.c_void_p * 1)(got.ctypes.data)
        assert L.nkv_group_roots_allgather(grp.h, bad, None, _lib.p8(got)) == _lib.NKV_ERR_INVALID
        # one tree through the split entry (g = 1: member 0 holds every leaf)
        base, off, ln = ragged(5003, 11)
        nodes = np.zeros((L.nkv_total_nodes(5003), 20), np.uint8)
        img = np.zeros(L.nkv_bfs_size(5003), np.uint8)
        root = np.zeros(20, np.uint8)
        _lib.check(L.nkv_group_tree_from_values(grp.h, _lib.p8(base), _lib.p64(off), _lib.p64(ln), 5003,
                                                _lib.p8(root), _lib.p8(nodes), _lib.p8(img)))
        want = want_tree(oracle, base, off, ln)
        assert np.array_equal(nodes, want) and root.tobytes() == want[-1].tobytes()
        assert img.tobytes() == oracle.bfs_image(want, 5003)


def split_parts(_lib, g, n, data, L):
    """Member r's strided leaf range [r span, ...) of n leaves of L bytes (device tensors)."""
    span = _lib.lib().nkv_split_span(n, g)
    parts, keep = [], []
    for r in range(g):
        lo, hi = min(n, r * span), min(n, (r + 1) * span)
        if hi > lo:
            d = dev(data[lo * L:hi * L])
            keep.append(d)
            parts.append(_lib.table(_lib.NKV_TABLE_STRIDED, 0, hi - lo, base=d.data_ptr(), stride=L, length=L))
        else:
            parts.append(_lib.table(_lib.NKV_TABLE_STRIDED, 0, 0))
    return parts, keep


@pytest.mark.parametrize("g", [2, 3, 4])
@pytest.mark.parametrize("n", [1, 2, 3, 5, 64, 65, 1000, 4097, 65537])
def test_group_split_tree_copy_transport(nkv, oracle, g, n):
    """One tree over g members (device 0 listed g times: copy transport) against
    the oracle: root, every level (nkv_group_tree_fetch) and the Serialize image."""
    _lib, _ = nkv
    L = _lib.lib()
    vl = 100
    data = np.frombuffer(np.random.default_rng(n * 7 + g).bytes(n * vl), np.uint8).copy()
    want = oracle.tree_from_digests(oracle.leaf_hashes_strided(data, vl, vl, n))
    with _lib.Group([0] * g) as grp:
        assert grp.transport == _lib.NKV_TRANSPORT_COPY
        parts, keep = split_parts(_lib, g, n, data, vl)
        arr = (_lib.NkvTable * g)(*parts)
        root = np.zeros(20, np.uint8)
        d_roots = [torch.zeros(20, dtype=torch.uint8, device="cuda") for _ in range(g)]
        _lib.check(L.nkv_group_tree_dev(grp.h, arr, n, (ctypes.c_void_p * g)(*[d.data_ptr() for d in d_roots]),
                                        _lib.p8(root)))
        assert root.tobytes() == want[-1].tobytes()
        # every member reduced the top levels and holds the root
        assert all(d.cpu().numpy().tobytes() == want[-1].tobytes() for d in d_roots)
        nodes = np.zeros((L.nkv_total_nodes(n), 20), np.uint8)
        img = np.zeros(L.nkv_bfs_size(n), np.uint8)
        _lib.check(L.nkv_group_tree_fetch(grp.h, _lib.p8(nodes), _lib.p8(img)))
        assert np.array_equal(nodes, want)
        assert img.tobytes() == oracle.bfs_image(want, n)
        # a part whose length does not match the plan is refused
        if n > 1:
            bad = list(parts)
            bad[0] = _lib.table(_lib.NKV_TABLE_STRIDED, 0, parts[0].n - 1, base=parts[0].base, stride=vl, length=vl)
            assert L.nkv_group_tree_dev(grp.h, (_lib.NkvTable * g)(*bad), n, None, None) == _lib.NKV_ERR_INVALID
            # the refused call left no tree behind -- fetch refuses
            # instead of reading the previous tree's buffers with a new plan
            assert L.nkv_group_tree_fetch(grp.h, _lib.p8(nodes), _lib.p8(img)) == _lib.NKV_ERR_INVALID
        # a good split, then a refused one with a larger n, then fetch
        _lib.check(L.nkv_group_tree_dev(grp.h, arr, n, None, _lib.p8(root)))
        assert L.nkv_group_tree_dev(grp.h, arr, 4 * n + 3, None, None) == _lib.NKV_ERR_INVALID
        assert L.nkv_group_tree_fetch(grp.h, _lib.p8(nodes), _lib.p8(img)) == _lib.NKV_ERR_INVALID
        # a member's root buffer on another device (host memory) is refused
        droot_bad = (ctypes.c_void_p * g)(*([0] * (g - 1) + [root.ctypes.data]))
        assert L.nkv_group_tree_dev(grp.h, arr, n, droot_bad, None) == _lib.NKV_ERR_INVALID


def test_group_split_refusals_leave_no_tree(nkv, oracle):
    """after any refused or failed split call -- the device form with a
    part of the wrong length, with n = 0, or the host form with a null pointer --
    nkv_group_tree_fetch refuses; a good call after it fetches the new tree.
    d_roots may be NULL or hold NULL entries."""
    _lib, _ = nkv
    L = _lib.lib()
    g, n, vl = 3, 1000, 64
    data = np.frombuffer(np.random.default_rng(44).bytes(n * vl), np.uint8).copy()
    want = oracle.tree_from_digests(oracle.leaf_hashes_strided(data, vl, vl, n))
    nodes = np.zeros((L.nkv_total_nodes(n), 20), np.uint8)
    with _lib.Group([0] * g) as grp:
        parts, keep = split_parts(_lib, g, n, data, vl)
        arr = (_lib.NkvTable * g)(*parts)
        one = torch.zeros(20, dtype=torch.uint8, device="cuda")
        roots = (ctypes.c_void_p * g)(None, one.data_ptr(), None)  # only member 1 wants its root
        for bad in (lambda: L.nkv_group_tree_dev(grp.h, arr, n + 1, None, None),
                    lambda: L.nkv_group_tree_dev(grp.h, arr, 0, None, None),
                    lambda: L.nkv_group_tree_from_values(grp.h, None, None, None, n, None, None, None)):
            _lib.check(L.nkv_group_tree_dev(grp.h, arr, n, roots, None))
            grp.sync()
            assert one.cpu().numpy().tobytes() == want[-1].tobytes()
            assert bad() != _lib.NKV_OK
            assert L.nkv_group_tree_fetch(grp.h, _lib.p8(nodes), None) == _lib.NKV_ERR_INVALID
        _lib.check(L.nkv_group_tree_dev(grp.h, arr, n, None, None))
        _lib.check(L.nkv_group_tree_fetch(grp.h, _lib.p8(nodes), None))
        assert np.array_equal(nodes, want)


def values_parts(_lib, g, n, base, off, ln):
    """Member r's ragged leaf range as a VALUES table: its values' bytes, offsets
    rebased to them, lengths (device tensors)."""
    span = _lib.lib().nkv_split_span(n, g)
    parts, keep = [], []
    for r in range(g):
        lo, hi = min(n, r * span), min(n, (r + 1) * span)
        if hi > lo:
            b0 = int(off[lo])
            b1 = int(off[hi - 1] + ln[hi - 1])
            db = dev(np.concatenate([base[b0:b1], np.zeros(1, np.uint8)]))
            do, dl = dev((off[lo:hi] - b0).view(np.int64)), dev(ln[lo:hi].view(np.int64))
            keep += [db, do, dl]
            parts.append(_lib.table(_lib.NKV_TABLE_VALUES, 0, hi - lo, base=db.data_ptr(), off=do.data_ptr(),
                                    lens=dl.data_ptr()))
        else:
            parts.append(_lib.table(_lib.NKV_TABLE_VALUES, 0, 0))
    return parts, keep


@pytest.mark.parametrize("seed", range(12))
def test_group_split_fuzz_values(nkv, oracle, seed):
    """Seeded fuzz of the split: n log-uniform in [1, 2^18], g in 1..8 (device 0
    repeated: copy transport; g = 1 also), ragged unaligned values 0-299 bytes;
    root, every level and the image against the oracle."""
    _lib, _ = nkv
    L = _lib.lib()
    rng = np.random.default_rng(1000 + seed)
    n = int(np.exp(rng.uniform(0, np.log(1 << 18))))
    n = max(1, n)
    g = int(rng.integers(1, 9))
    base, off, ln = ragged(n, 2000 + seed)
    want = want_tree(oracle, base, off, ln)
    with _lib.Group([0] * g) as grp:
        parts, keep = values_parts(_lib, g, n, base, off, ln)
        root = np.zeros(20, np.uint8)
        _lib.check(L.nkv_group_tree_dev(grp.h, (_lib.NkvTable * g)(*parts), n, None, _lib.p8(root)))
        assert root.tobytes() == want[-1].tobytes(), (n, g)
        nodes = np.zeros((L.nkv_total_nodes(n), 20), np.uint8)
        img = np.zeros(L.nkv_bfs_size(n), np.uint8)
        _lib.check(L.nkv_group_tree_fetch(grp.h, _lib.p8(nodes), _lib.p8(img)))
        assert np.array_equal(nodes, want), (n, g)
        assert img.tobytes() == oracle.bfs_image(want, n), (n, g)


@pytest.mark.parametrize("g", [2, 4])
def test_group_host_forms_copy_transport(nkv, oracle, g):
    """nkv_group_tree_from_values (one tree, one host thread per member) and
    nkv_group_trees_from_values (k tables round-robin) from host memory."""
    _lib, _ = nkv
    L = _lib.lib()
    with _lib.Group([0] * g) as grp:
        for n in (1, 7, 3001, 70001):
            base, off, ln = ragged(n, n)
            want = want_tree(oracle, base, off, ln)
            root = np.zeros(20, np.uint8)
            nodes = np.zeros((L.nkv_total_nodes(n), 20), np.uint8)
            img = np.zeros(L.nkv_bfs_size(n), np.uint8)
            _lib.check(L.nkv_group_tree_from_values(grp.h, _lib.p8(base), _lib.p64(off), _lib.p64(ln), n,
                                                    _lib.p8(root), _lib.p8(nodes), _lib.p8(img)))
            assert root.tobytes() == want[-1].tobytes()
            assert np.array_equal(nodes, want)
            assert img.tobytes() == oracle.bfs_image(want, n)
        k = 5
        vals = [ragged(1000 + 37 * t, 100 + t) for t in range(k)]
        roots = [np.zeros(20, np.uint8) for _ in range(k)]
        tabs = (_lib.NkvValues * k)(*[
            _lib.NkvValues(v[0].ctypes.data, v[1].ctypes.data, v[2].ctypes.data, len(v[1]), r.ctypes.data, None, None)
            for v, r in zip(vals, roots)])
        _lib.check(L.nkv_group_trees_from_values(grp.h, tabs, k))
        for v, r in zip(vals, roots):
            assert r.tobytes() == want_tree(oracle, *v)[-1].tobytes()


def test_group_trees_dev_copy_transport_roots_in_table_order(nkv, oracle):
    _lib, _ = nkv
    L = _lib.lib()
    k, g = 7, 3
    with _lib.Group([0] * g) as grp:
        keep, tabs, wants = [], [], []
        for t in range(k):
            n = 500 + 101 * t
            data = np.frombuffer(np.random.default_rng(t).bytes(n * 256), np.uint8).copy()
            d, nb = dev(data), nodes_buf(L, n)
            keep += [d, nb]
            tabs.append(_lib.table(_lib.NKV_TABLE_STRIDED, nb.data_ptr(), n, base=d.data_ptr(), stride=256,
                                   length=256))
            wants.append(oracle.tree_from_digests(oracle.leaf_hashes_strided(data, 256, 256, n))[-1].tobytes())
        roots = np.zeros(k * 20, np.uint8)
        _lib.check(L.nkv_group_trees_dev(grp.h, (_lib.NkvTable * k)(*tabs), k, _lib.p8(roots)))
        assert [roots[20 * t:20 * t + 20].tobytes() for t in range(k)] == wants
        # a table on the wrong device (host memory) is refused before any launch
        host = np.zeros(4096, np.uint8)
        bad = list(tabs)
        bad[1] = _lib.table(_lib.NKV_TABLE_STRIDED, host.ctypes.data, 16, base=keep[0].data_ptr(), stride=256,
                            length=256)
        assert L.nkv_group_trees_dev(grp.h, (_lib.NkvTable * k)(*bad), k, None) == _lib.NKV_ERR_INVALID


def test_group_roots_allgather_copy_transport(nkv):
    """The bare all-gather over the copy transport (device 0 listed 3 times):
    every member's 20 bytes land on every member in member order, through the
    caller's output buffers and through the group's own."""
    _lib, _ = nkv
    L = _lib.lib()
    g = 3
    with _lib.Group([0] * g) as grp:
        src = [torch.arange(20 * r, 20 * r + 20, dtype=torch.uint8, device="cuda") for r in range(g)]
        outs = [torch.zeros(20 * g, dtype=torch.uint8, device="cuda") for _ in range(g)]
        want = b"".join(x.cpu().numpy().tobytes() for x in src)
        got = np.zeros(20 * g, np.uint8)
        _lib.check(L.nkv_group_roots_allgather(grp.h, (ctypes.c_void_p * g)(*[x.data_ptr() for x in src]),
                                               (ctypes.c_void_p * g)(*[o.data_ptr() for o in outs]), _lib.p8(got)))
        assert got.tobytes() == want
        assert all(o.cpu().numpy().tobytes() == want for o in outs)
        got[:] = 0
        _lib.check(L.nkv_group_roots_allgather(grp.h, (ctypes.c_void_p * g)(*[x.data_ptr() for x in src]), None,
                                               _lib.p8(got)))
        assert got.tobytes() == want


def test_stream_handover_orders_records_calls(nkv, oracle):
    """an asynchronous verify call on stream A, the next on
    stream B at once; the pass flags one call leaves for the next stay ordered."""
    _lib, ctx = nkv
    L = _lib.lib()
    s, ro, vo, vl = records(8192, 1500, 21)
    s2 = s.copy().reshape(8192, -1)
    s2[100, 40] ^= 1  # one bad Crc in the second table
    ds, ds2, dr = dev(s), dev(s2.reshape(-1)), dev(ro.view(np.int64))
    n1, n2 = nodes_buf(L, 8192), nodes_buf(L, 8192)
    st1 = torch.zeros(3, dtype=torch.int64, device="cuda")
    st2 = torch.zeros(3, dtype=torch.int64, device="cuda")
    a, b = torch.cuda.Stream(), torch.cuda.Stream()
    for _ in range(3):
        ctx.set_stream(a.cuda_stream)
        _lib.check(L.nkv_tree_verify_records_dev(ctx.h, ds.data_ptr(), s.size, dr.data_ptr(), 8192, n1.data_ptr(),
                                                 None, st1.data_ptr()))
        ctx.set_stream(b.cuda_stream)
        _lib.check(L.nkv_tree_verify_records_dev(ctx.h, ds2.data_ptr(), s.size, dr.data_ptr(), 8192,
                                                 n2.data_ptr(), None, st2.data_ptr()))
    torch.cuda.synchronize()
    ctx.set_stream(torch.cuda.current_stream().cuda_stream)
    assert np.array_equal(host_nodes(n1), want_tree(oracle, s, vo, vl))
    assert np.array_equal(host_nodes(n2), want_tree(oracle, s2.reshape(-1), vo, vl))
    assert st1.cpu().tolist() == [0, -1, 0]
    assert st2.cpu().tolist() == [1, 100, 0]


def test_pinned_arena_zero_copy_and_streaming(nkv, oracle):
    """Values inside an nkv_host_alloc block go to the device in one DMA straight
    from the block; nkv_host_stream queues a settled prefix ahead of the call;
    a smaller upto starts a new batch.  Aligned and unaligned places."""
    _lib, ctx = nkv
    L = _lib.lib()
    cap = 8 << 20
    p = ctypes.c_void_p()
    _lib.check(L.nkv_host_alloc(ctx.h, cap, ctypes.byref(p)))
    try:
        arena = np.ctypeslib.as_array((ctypes.c_uint8 * cap).from_address(p.value))
        for batch, (n, pad) in enumerate([(2000, 16), (1500, 1), (3000, 16)]):
            rng = np.random.default_rng(batch)
            ln = rng.integers(0, 2000, n).astype(np.uint64)
            off = np.zeros(n, np.uint64)
            pos = 0
            for i in range(n):
                off[i] = pos
                pos += int(ln[i])
                pos = (pos + pad - 1) // pad * pad
            arena[:pos] = np.frombuffer(rng.bytes(pos), np.uint8)
            # stream the first half ahead (as NewLeaf would, chunk by chunk)
            _lib.check(L.nkv_host_stream(ctx.h, p, pos // 2))
            _lib.check(L.nkv_host_stream(ctx.h, p, pos // 2 + 4096))
            want = want_tree(oracle, arena[:pos].copy(), off, ln)
            root = np.zeros(20, np.uint8)
            nodes = np.zeros((L.nkv_total_nodes(n), 20), np.uint8)
            _lib.check(L.nkv_tree_from_values(ctx.h, ctypes.cast(p, _lib._u8p), _lib.p64(off), _lib.p64(ln), n,
                                              _lib.p8(root), _lib.p8(nodes), None))
            assert np.array_equal(nodes, want) and root.tobytes() == want[-1].tobytes()
            # NewLeaf digests alone from the same block (base inside the block)
            out = np.zeros((n, 20), np.uint8)
            _lib.check(L.nkv_leaf_hash(ctx.h, ctypes.cast(p, _lib._u8p), _lib.p64(off), _lib.p64(ln), n, _lib.p8(out)))
            assert np.array_equal(out, want[:n])
        # an upto past the block, or a pointer that is no block of this context
        assert L.nkv_host_stream(ctx.h, p, cap + 1) == _lib.NKV_ERR_INVALID
        other = np.zeros(64, np.uint8)
        assert L.nkv_host_stream(ctx.h, other.ctypes.data, 10) == _lib.NKV_ERR_INVALID
    finally:
        _lib.check(L.nkv_host_free(ctx.h, p))


def test_host_call_timing_and_clock_probe(nkv, oracle):
    _lib, ctx = nkv
    L = _lib.lib()
    n, vl = 65536, 4096
    d = torch.empty(n * vl, dtype=torch.uint8, device="cuda")
    ctx.set_stream(torch.cuda.current_stream().cuda_stream)
    _lib.check(L.nkv_fill_splitmix64_dev(ctx.h, d.data_ptr(), n * vl, 5))
    nb = nodes_buf(L, n)
    ctx.set_timing(True, clock=True)
    try:
        for _ in range(3):
            _lib.check(L.nkv_tree_from_strided_dev(ctx.h, d.data_ptr(), vl, vl, n, nb.data_ptr()))
        mhz, waves = ctx.clock()
        assert 300.0 < mhz < 3500.0, mhz
        assert waves == 3 * n // 64
        # upload / kernels / download of a host call
        base, off, ln = ragged(5000, 9)
        root = np.zeros(20, np.uint8)
        _lib.check(L.nkv_tree_from_values(ctx.h, _lib.p8(base), _lib.p64(off), _lib.p64(ln), 5000, _lib.p8(root),
                                          None, None))
        a, b, c = ctypes.c_float(), ctypes.c_float(), ctypes.c_float()
        _lib.check(L.nkv_ctx_last_host_timing(ctx.h, ctypes.byref(a), ctypes.byref(b), ctypes.byref(c)))
        assert a.value >= 0 and b.value > 0 and c.value >= 0
        assert root.tobytes() == want_tree(oracle, base, off, ln)[-1].tobytes()
    finally:
        ctx.set_timing(False)
    want = oracle.tree_from_digests(oracle.leaf_hashes_strided(d.cpu().numpy(), vl, vl, n, threads=8))
    assert nb[-20:].cpu().numpy().tobytes() == want[-1].tobytes()


def test_timing_every_kth_call(nkv, oracle):
    """NKV_OPT_TIMING_EVERY k: only calls 0, k, 2k, ... since set_timing record
    events (the timed loop's sampling); out-of-range k refused; results unchanged."""
    _lib, ctx = nkv
    L = _lib.lib()
    n, vl = 20000, 256
    d = torch.empty(n * vl, dtype=torch.uint8, device="cuda")
    ctx.set_stream(torch.cuda.current_stream().cuda_stream)
    _lib.check(L.nkv_fill_splitmix64_dev(ctx.h, d.data_ptr(), n * vl, 11))
    nb = nodes_buf(L, n)
    assert L.nkv_ctx_set_option(ctx.h, _lib.NKV_OPT_TIMING_EVERY, 0) == _lib.NKV_ERR_INVALID
    try:
        for k, calls, want_sampled in ((3, 7, 3), (1, 4, 4), (8, 20, 3)):
            ctx.set_option(_lib.NKV_OPT_TIMING_EVERY, k)
            ctx.set_timing(True)
            for _ in range(calls):
                _lib.check(L.nkv_tree_from_strided_dev(ctx.h, d.data_ptr(), vl, vl, n, nb.data_ptr()))
            got, leaf_ms, reduce_ms = ctx.timing_summary()
            assert got == want_sampled, (k, got)
            assert leaf_ms > 0 and reduce_ms > 0
            # a host call that is not sampled has no host timing; a sampled one has
            ctx.set_option(_lib.NKV_OPT_TIMING_EVERY, 2)
            ctx.set_timing(True)
            base, off, ln = ragged(3000, 4)
            root = np.zeros(20, np.uint8)
            a, b, c = ctypes.c_float(), ctypes.c_float(), ctypes.c_float()
            for i in range(3):
                _lib.check(L.nkv_tree_from_values(ctx.h, _lib.p8(base), _lib.p64(off), _lib.p64(ln), 3000,
                                                  _lib.p8(root), None, None))
                rc = L.nkv_ctx_last_host_timing(ctx.h, ctypes.byref(a), ctypes.byref(b), ctypes.byref(c))
                assert rc == (_lib.NKV_OK if i % 2 == 0 else _lib.NKV_ERR_INVALID), (i, rc)
            assert root.tobytes() == want_tree(oracle, base, off, ln)[-1].tobytes()
    finally:
        ctx.set_timing(False)
        ctx.set_option(_lib.NKV_OPT_TIMING_EVERY, 1)
    want = oracle.tree_from_digests(oracle.leaf_hashes_strided(d.cpu().numpy(), vl, vl, n, threads=8))
    assert nb[-20:].cpu().numpy().tobytes() == want[-1].tobytes()


def test_python_mirror_serialize_reads_the_live_tree(nkv, oracle):
    """merkletree.go:75-89 walks the live tree: after New, a leaf's and an
    interior node's Data changed through Root show in the image exactly as the
    literal restatement's walk writes them."""
    from nakevaleng_amd import merkletree as mt
    from oracle import merkle_ref as ref
    for n in (1, 2, 37, 1000):
        data = oracle.splitmix64_bytes(n * 50, 0xAB + n)
        vals = [data[50 * i:50 * i + 50].tobytes() for i in range(n)]
        t = mt.New([mt.NewLeaf(v) for v in vals])
        r = ref.New([ref.NewLeaf(v) for v in vals])
        assert t.SerializeBytes() == r.SerializeBytes()  # untouched
        for tree in (t, r):
            leaf = tree.Root
            while leaf.Left is not None:
                leaf = leaf.Left
            leaf.Data = bytes([0xAB]) * 20
            d = tree.Root.Data
            tree.Root.Data = bytes([d[0] ^ 0xFF]) + bytes(d[1:])
        assert t.SerializeBytes() == r.SerializeBytes()


def test_pruned_variants_are_refused(nkv):
    """only the surviving paths are selectable -- LEAF_LOAD 4
    (register runs) / 11 (staged), the work-queue kernel with its 3-slot ring."""
    _lib, ctx = nkv
    L = _lib.lib()
    for v in (0, 1, 2, 3, 5, 6, 7, 8, 9, 10, 12):
        assert L.nkv_ctx_set_option(ctx.h, _lib.NKV_OPT_LEAF_LOAD, v) == _lib.NKV_ERR_INVALID
    for v in (4, 11):
        assert L.nkv_ctx_set_option(ctx.h, _lib.NKV_OPT_LEAF_LOAD, v) == _lib.NKV_OK
    # the retired DEEP_PREFETCH and QUEUE_RING keys accept their only value
    # until an ABI version bump, and nothing else
    for key, only in ((3, 3), (9, 13)):
        for v in (0, 1, 4, 12, 14):
            assert L.nkv_ctx_set_option(ctx.h, key, v) == _lib.NKV_ERR_INVALID
        assert L.nkv_ctx_set_option(ctx.h, key, only) == _lib.NKV_OK
    # round 6: the pair kernel NKV_OPT_QUEUE_PAIR selected is gone (it failed
    # its first GPU parity run); the key accepts only 0
    for v in (1, 50, 80, 100, -1):
        assert L.nkv_ctx_set_option(ctx.h, _lib.NKV_OPT_QUEUE_PAIR, v) == _lib.NKV_ERR_INVALID
    assert L.nkv_ctx_set_option(ctx.h, _lib.NKV_OPT_QUEUE_PAIR, 0) == _lib.NKV_OK
    for v in (0, 4, 5):
        assert L.nkv_ctx_set_option(ctx.h, _lib.NKV_OPT_QUEUE_WAVES, v) == _lib.NKV_ERR_INVALID
    assert L.nkv_ctx_set_option(ctx.h, _lib.NKV_OPT_QUEUE_WAVES, 3) == _lib.NKV_OK
    for v in (1, 2, 9, 10):  # the CRC kernel: lane-private tables (0) or the span groups (8)
        assert L.nkv_ctx_set_option(ctx.h, _lib.NKV_OPT_CRC_LOAD, v) == _lib.NKV_ERR_INVALID
    for v in (0, 9):
        assert L.nkv_ctx_set_option(ctx.h, _lib.NKV_OPT_TABLE_LANES, v) == _lib.NKV_ERR_INVALID
    ctx.set_option(_lib.NKV_OPT_TABLE_LANES, 2)
    ctx.set_option(_lib.NKV_OPT_LEAF_LOAD, 4)
