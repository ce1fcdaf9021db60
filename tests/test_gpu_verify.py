"""GPU: the compaction read in one call (nkv_tree_verify_records_dev) -- the
Merkle tree of the records' Values (merklenode.go:27-34, merkletree.go:31-64)
and record.Deserialize's checksum check (record.go:163-169) -- against the C
oracle.  Similar-size batches take the fused kernel (k_leaf_verify), ragged ones
the checksum kernel plus the length-sorted leaf kernel; both must agree with
the oracle bit for bit, corrupted records and bad headers included."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SEED = 0x6E616B65


def _torch():
    import torch
    return torch


def _dev(torch, a):
    return torch.from_numpy(np.ascontiguousarray(a).view(np.uint8).copy()).cuda()


def _stream(rng, n, kmax=40, vmax=3000):
    from nakevaleng_amd import record
    recs = [record.New(rng.integers(0, 256, int(k), dtype=np.uint8).tobytes(),
                       rng.integers(0, 256, int(v), dtype=np.uint8).tobytes(), timestamp=1)
            for k, v in zip(rng.integers(0, kmax + 1, n), rng.integers(0, vmax + 1, n))]
    stream, sizes = record.data_table(recs)
    off = np.zeros(n, np.uint64)
    off[1:] = np.cumsum(sizes[:-1])
    return np.frombuffer(stream, np.uint8).copy(), off


def _sstable(n, ks=16, vs=4050, oracle=None):
    """n records of TotalSize 30 + ks + vs with correct stored checksums."""
    rb = 30 + ks + vs
    body = oracle.splitmix64_bytes(n * rb, SEED).reshape(n, rb)
    body[:, 4:14] = 0
    body[:, 14:22] = np.frombuffer(np.uint64(ks).tobytes(), np.uint8)
    body[:, 22:30] = np.frombuffer(np.uint64(vs).tobytes(), np.uint8)
    off = np.arange(n, dtype=np.uint64) * rb
    crc, _, _ = oracle.record_crcs(body.reshape(-1), off)
    body[:, 0:4] = crc.view(np.uint8).reshape(n, 4)
    return body.reshape(-1).copy(), off


def _want(oracle, buf, off):
    """Oracle tree of the Values, checksums, ok flags, mismatch count (valid headers)."""
    n = off.size
    voff = np.zeros(n, np.uint64)
    vlen = np.zeros(n, np.uint64)
    for i, r in enumerate(off.tolist()):
        ks = int(buf[r + 14:r + 22].view(np.uint64)[0])
        voff[i], vlen[i] = r + 30 + ks, int(buf[r + 22:r + 30].view(np.uint64)[0])
    nodes = oracle.tree_from_digests(oracle.leaf_hashes(buf, voff, vlen, threads=8))
    crc, ok, bad = oracle.record_crcs(buf, off)
    return nodes, crc, ok, bad


def _run(torch, L, _lib, ctx, buf, off, want_crc=True):
    n = off.size
    d_buf, d_off = _dev(torch, buf), _dev(torch, off)
    d_nodes = torch.zeros(L.nkv_total_nodes(n) * 20, dtype=torch.uint8, device="cuda")
    d_crc = torch.zeros(n * 4, dtype=torch.uint8, device="cuda")
    d_stats = torch.zeros(24, dtype=torch.uint8, device="cuda")
    _lib.check(L.nkv_tree_verify_records_dev(ctx.h, d_buf.data_ptr(), buf.size, d_off.data_ptr(), n,
                                             d_nodes.data_ptr(), d_crc.data_ptr() if want_crc else None,
                                             d_stats.data_ptr()))
    torch.cuda.synchronize()
    return (d_nodes.cpu().numpy().reshape(-1, 20), d_crc.cpu().numpy().view(np.uint32),
            d_stats.cpu().numpy().view(np.uint64).tolist())


def _check(got, want, n):
    nodes, crc, stats = got
    w_nodes, w_crc, w_ok, w_bad = want
    assert np.array_equal(nodes, w_nodes)
    assert np.array_equal(crc, w_crc)
    bad_idx = [i for i in range(n) if not w_ok[i]]
    assert stats[0] == w_bad == len(bad_idx)
    assert stats[1] == (bad_idx[0] if bad_idx else 2**64 - 1)
    assert stats[2] == 0


@pytest.mark.parametrize("bucket", [2, 0, 1])
def test_verify_sstable_shape(nkv, oracle, bucket):
    """64 Ki SSTable records (16-B key, 4,050-B value): the fused kernel under
    auto order and forced input order, the split path under forced sorting."""
    torch = _torch()
    _lib, ctx = nkv
    ctx.set_stream(torch.cuda.current_stream().cuda_stream)
    ctx.set_option(_lib.NKV_OPT_BUCKET, bucket)
    L = _lib.lib()
    n = 1 << 16
    buf, off = _sstable(n, oracle=oracle)
    rng = np.random.default_rng(3)
    for i in sorted(set(rng.integers(0, n, 40).tolist())):  # key, value and tail bytes
        buf[int(off[i]) + 30 + int(rng.integers(0, 16 + 4050))] ^= 0x10
    try:
        got = _run(torch, L, _lib, ctx, buf, off)
    finally:
        ctx.set_option(_lib.NKV_OPT_BUCKET, 2)
    _check(got, _want(oracle, buf, off), n)


@pytest.mark.parametrize("bucket", [2, 0])
@pytest.mark.parametrize("n", [1, 2, 63, 64, 65, 257, 3000, 5000])
def test_verify_ragged_records(nkv, oracle, n, bucket):
    """Keys 0-40 B and values 0-9,000 B at every alignment; auto order sorts
    them (split path), forced input order runs them through the fused kernel."""
    torch = _torch()
    _lib, ctx = nkv
    ctx.set_stream(torch.cuda.current_stream().cuda_stream)
    ctx.set_option(_lib.NKV_OPT_BUCKET, bucket)
    L = _lib.lib()
    rng = np.random.default_rng(n)
    buf, off = _stream(rng, n, vmax=9000)
    for i in sorted(set(rng.integers(0, n, max(1, n // 50)).tolist())) if n > 1 else []:
        buf[int(off[i])] ^= 0x01  # the stored Crc itself
    try:
        got = _run(torch, L, _lib, ctx, buf, off)
    finally:
        ctx.set_option(_lib.NKV_OPT_BUCKET, 2)
    _check(got, _want(oracle, buf, off), n)


@pytest.mark.parametrize("n", [5000, 8192])
def test_verify_header_outside_stream(nkv, oracle, n):
    """A ValueSize past the stream: stats[2] is set, that leaf hashes the empty
    value, every other record is still checked and hashed."""
    import hashlib
    torch = _torch()
    _lib, ctx = nkv
    ctx.set_stream(torch.cuda.current_stream().cuda_stream)
    L = _lib.lib()
    buf, off = _sstable(n, ks=16, vs=1000, oracle=oracle)
    voff = off + 46
    leaves = oracle.leaf_hashes(buf, voff, np.full(n, 1000, np.uint64), threads=8)
    j = n // 3
    leaves[j] = np.frombuffer(hashlib.sha1(b"").digest(), np.uint8)
    buf[int(off[j]) + 22:int(off[j]) + 30] = np.frombuffer(np.uint64(1 << 40).tobytes(), np.uint8)
    nodes, _, stats = _run(torch, L, _lib, ctx, buf, off, want_crc=False)
    assert np.array_equal(nodes, oracle.tree_from_digests(leaves))
    assert stats == [0, 2**64 - 1, 1]


def test_verify_matches_separate_calls(nkv, oracle):
    """Same tree as nkv_tree_from_records_dev and same checksums/stats as
    nkv_record_crc_dev on one stream."""
    torch = _torch()
    _lib, ctx = nkv
    ctx.set_stream(torch.cuda.current_stream().cuda_stream)
    L = _lib.lib()
    n = 20000
    buf, off = _sstable(n, ks=24, vs=2000, oracle=oracle)
    buf[int(off[777]) + 100] ^= 0x80
    nodes, crc, stats = _run(torch, L, _lib, ctx, buf, off)
    d_buf, d_off = _dev(torch, buf), _dev(torch, off)
    d_nodes = torch.zeros(L.nkv_total_nodes(n) * 20, dtype=torch.uint8, device="cuda")
    d_err = torch.zeros(1, dtype=torch.int32, device="cuda")
    _lib.check(L.nkv_tree_from_records_dev(ctx.h, d_buf.data_ptr(), buf.size, d_off.data_ptr(), n,
                                           d_nodes.data_ptr(), d_err.data_ptr()))
    d_crc = torch.zeros(n * 4, dtype=torch.uint8, device="cuda")
    d_stats = torch.zeros(24, dtype=torch.uint8, device="cuda")
    _lib.check(L.nkv_record_crc_dev(ctx.h, d_buf.data_ptr(), buf.size, d_off.data_ptr(), n, d_crc.data_ptr(),
                                    d_stats.data_ptr()))
    torch.cuda.synchronize()
    assert np.array_equal(nodes, d_nodes.cpu().numpy().reshape(-1, 20))
    assert np.array_equal(crc, d_crc.cpu().numpy().view(np.uint32))
    assert stats == d_stats.cpu().numpy().view(np.uint64).tolist() == [1, 777, 0]


def test_pass_flag_sets_alternate(nkv, oracle):
    """The records entries keep their deferred-pass flags in two per-context
    sets used by alternate calls, each call resetting the other set: a sequence
    of verify and plain records calls on one context, good / corrupted / bad
    header / ragged (deferred) / small (all sorted) tables in an order that puts
    every case on both sets, each checked against the oracle."""
    import hashlib
    torch = _torch()
    _lib, ctx = nkv
    ctx.set_stream(torch.cuda.current_stream().cuda_stream)
    L = _lib.lib()
    cases = {}
    buf, off = _sstable(5000, ks=16, vs=1000, oracle=oracle)
    cases["good"] = (buf, off, _want(oracle, buf, off), 0)
    bad = buf.copy()
    for i in (3, 700, 4999):
        bad[int(off[i]) + 30 + 16 + 5] ^= 0x40  # value byte: stored Crc mismatch
    cases["crc"] = (bad, off, _want(oracle, bad, off), 0)
    hdr = buf.copy()
    j = 1234
    hdr[int(off[j]) + 22:int(off[j]) + 30] = np.frombuffer(np.uint64(1 << 40).tobytes(), np.uint8)
    leaves = oracle.leaf_hashes(buf, off + 46, np.full(off.size, 1000, np.uint64), threads=8)
    leaves[j] = np.frombuffer(hashlib.sha1(b"").digest(), np.uint8)
    cases["header"] = (hdr, off, None, 1, oracle.tree_from_digests(leaves))
    rng = np.random.default_rng(77)
    rbuf, roff = _stream(rng, 5000, vmax=9000)
    rbuf[int(roff[10])] ^= 0x01
    cases["ragged"] = (rbuf, roff, _want(oracle, rbuf, roff), 0)
    sbuf, soff = _stream(rng, 3000, vmax=5000)
    cases["small"] = (sbuf, soff, _want(oracle, sbuf, soff), 0)
    order = ["good", "header", "good", "ragged", "crc", "good", "small", "header", "ragged", "good", "good",
             "crc", "header", "small", "good"]
    for step, name in enumerate(order):
        case = cases[name]
        buf_, off_, want, herr = case[:4]
        n = off_.size
        if step % 3 == 2:  # a plain records call between the verify calls
            d_buf, d_off = _dev(torch, buf_), _dev(torch, off_)
            d_nodes = torch.zeros(L.nkv_total_nodes(n) * 20, dtype=torch.uint8, device="cuda")
            d_err = torch.full((1,), 7, dtype=torch.int32, device="cuda")
            _lib.check(L.nkv_tree_from_records_dev(ctx.h, d_buf.data_ptr(), buf_.size, d_off.data_ptr(), n,
                                                   d_nodes.data_ptr(), d_err.data_ptr()))
            torch.cuda.synchronize()
            assert int(d_err.item()) == herr, (step, name)
            w_nodes = case[4] if want is None else want[0]
            assert np.array_equal(d_nodes.cpu().numpy().reshape(-1, 20), w_nodes), (step, name)
            continue
        got = _run(torch, L, _lib, ctx, buf_, off_, want_crc=want is not None)
        if want is None:
            assert np.array_equal(got[0], case[4]), (step, name)
            assert got[2] == [0, 2**64 - 1, 1], (step, name)
        else:
            _check(got, want, n)


@pytest.mark.parametrize("rec,ks", [(4096, 16), (1024, 16), (1024, 50), (256, 0), (384, 7), (192, 16), (4096, 97)])
def test_line_register_path_records(nkv, oracle, rec, ks):
    """Records whose segment 0 starts a 128-byte line (rec a multiple of 128)
    take the whole-line register path in k_leaf_records and k_leaf_verify;
    rec = 192 mixes line parities inside a wave (the segment stage instead).
    The last record ends at the end of the stream.  Both entries against the
    oracle, a few stored Crcs corrupted."""
    torch = _torch()
    _lib, ctx = nkv
    ctx.set_stream(torch.cuda.current_stream().cuda_stream)
    L = _lib.lib()
    n = 5000
    buf, off = _sstable(n, ks=ks, vs=rec - 30 - ks, oracle=oracle)
    assert buf.size == n * rec
    for i in (0, 777, n - 1):
        buf[int(off[i]) + 30 + ks] ^= 0x01  # first value byte
    want = _want(oracle, buf, off)
    _check(_run(torch, L, _lib, ctx, buf, off), want, n)
    d_buf, d_off = _dev(torch, buf), _dev(torch, off)
    d_nodes = torch.zeros(L.nkv_total_nodes(n) * 20, dtype=torch.uint8, device="cuda")
    d_err = torch.full((1,), 7, dtype=torch.int32, device="cuda")
    _lib.check(L.nkv_tree_from_records_dev(ctx.h, d_buf.data_ptr(), buf.size, d_off.data_ptr(), n,
                                           d_nodes.data_ptr(), d_err.data_ptr()))
    torch.cuda.synchronize()
    assert int(d_err.item()) == 0
    assert np.array_equal(d_nodes.cpu().numpy().reshape(-1, 20), want[0])
