"""GPU: the SSTable filter -- murmur3 Bloom inserts and
queries through the C-ABI, against the C oracle (pinned by the published
MurmurHash3_x86_32 vectors and scikit-learn's murmurhash3_32 in test_oracle.py).
Seeds are explicit (the reference draws them from the clock)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _torch():
    import torch
    return torch


def _dev(torch, a):
    return torch.from_numpy(np.ascontiguousarray(a).view(np.uint8).copy()).cuda()


def _keys(rng, n, lmax=40, gap=7):
    ln = rng.integers(0, lmax + 1, n).astype(np.uint64)
    off = np.zeros(n, np.uint64)
    off[1:] = np.cumsum(ln[:-1] + rng.integers(0, gap + 1, n - 1).astype(np.uint64))
    data = rng.integers(0, 256, int(off[-1] + ln[-1]) + 1, dtype=np.uint8)
    return data, off, ln


@pytest.mark.parametrize("m,k", [(1, 1), (31, 3), (1000, 7), (95851, 7), (10050663, 7), (5000, 20), (777, 0)])
def test_bloom_insert_device_matches_oracle(nkv, oracle, m, k):
    torch = _torch()
    _lib, ctx = nkv
    ctx.set_stream(torch.cuda.current_stream().cuda_stream)
    L = _lib.lib()
    rng = np.random.default_rng(m + k)
    data, off, ln = _keys(rng, 5000)
    ln[:4] = [1000, 4097, 3, 0]
    off = np.zeros_like(ln)
    off[1:] = np.cumsum(ln[:-1] + 3)
    data = rng.integers(0, 256, int(off[-1] + ln[-1]) + 1, dtype=np.uint8)
    seed0 = int(rng.integers(0, 2**32))
    words = ((m + 31) // 32) * 4
    d_bits = torch.zeros(words, dtype=torch.uint8, device="cuda")
    d_data, d_off, d_len = _dev(torch, data), _dev(torch, off), _dev(torch, ln)  # held until the kernel ran
    _lib.check(L.nkv_bloom_insert_dev(ctx.h, d_data.data_ptr(), d_off.data_ptr(), d_len.data_ptr(), ln.size,
                                      m, k, seed0, d_bits.data_ptr()))
    torch.cuda.synchronize()
    got = d_bits.cpu().numpy()
    want = oracle.bloom_insert(data, off, ln, m, k, seed0)
    assert np.array_equal(got[:want.size], want)
    assert not got[want.size:].any()


def test_bloom_query_device_matches_oracle(nkv, oracle):
    torch = _torch()
    _lib, ctx = nkv
    ctx.set_stream(torch.cuda.current_stream().cuda_stream)
    L = _lib.lib()
    rng = np.random.default_rng(3)
    data, off, ln = _keys(rng, 3000)
    m, k = oracle.bloom_params(3000, 0.05)
    bits = oracle.bloom_insert(data, off, ln, m, k, 99)
    qdata, qoff, qln = _keys(rng, 20000, lmax=12)
    words = np.zeros(((m + 31) // 32) * 4, np.uint8)
    words[:bits.size] = bits
    for d, o, l_ in ((data, off, ln), (qdata, qoff, qln)):
        out = torch.zeros(l_.size, dtype=torch.uint8, device="cuda")
        held = [_dev(torch, a) for a in (d, o, l_, words)]  # alive until the kernel ran
        _lib.check(L.nkv_bloom_query_dev(ctx.h, held[0].data_ptr(), held[1].data_ptr(), held[2].data_ptr(),
                                         l_.size, m, k, 99, held[3].data_ptr(), out.data_ptr()))
        torch.cuda.synchronize()
        assert np.array_equal(out.cpu().numpy().astype(bool), oracle.bloom_query(d, o, l_, m, k, 99, bits))


def test_bloom_from_records_and_mirror(nkv, oracle):
    from nakevaleng_amd import bloomfilter, record, sstable
    _lib, ctx = nkv
    rng = np.random.default_rng(4)
    recs = [record.New(rng.integers(0, 256, int(kk), dtype=np.uint8).tobytes(),
                       rng.integers(0, 256, int(v), dtype=np.uint8).tobytes(), timestamp=1)
            for kk, v in zip(rng.integers(1, 33, 2000), rng.integers(0, 300, 2000))]
    stream, sizes = record.data_table(recs)
    keys = [r.Key for r in recs]
    bf = sstable.make_filter_from_records(stream, sizes, seed=1234, ctx=ctx)
    kd = np.frombuffer(b"".join(keys), np.uint8)
    kl = np.array([len(x) for x in keys], np.uint64)
    ko = np.zeros_like(kl)
    ko[1:] = np.cumsum(kl[:-1])
    want = oracle.bloom_insert(kd, ko, kl, bf.M, bf.K, 1234)
    assert (bf.M, bf.K) == oracle.bloom_params(2000, 0.01)
    assert bf.HashSeeds == [1234 + j for j in range(bf.K)]
    assert bf.Contents == want.tobytes()
    bf2 = sstable.make_filter_contents(keys, seed=1234, ctx=ctx)
    assert bf2.Contents == want.tobytes()
    # the reference's Insert / Query shape (bloomfilter.go main(): true false true)
    b = bloomfilter.New(100, 0.2, seed=7, ctx=ctx)
    b.Insert(bytes([1, 2]))
    b.Insert(bytes([3, 4]))
    assert b.Query(bytes([1, 2])) and b.Query(bytes([3, 4]))
    assert b.Query(bytes([2, 5])) == bool(oracle.bloom_query(np.array([2, 5], np.uint8), np.zeros(1, np.uint64),
                                                             np.full(1, 2, np.uint64), b.M, b.K, 7,
                                                             np.frombuffer(b.Contents, np.uint8))[0])
    with pytest.raises(bloomfilter.BloomFilterError):
        bloomfilter.New(-1, 0.1)


def test_bloom_records_header_outside_stream(nkv):
    from nakevaleng_amd import record, sstable
    _lib, ctx = nkv
    recs = [record.New(b"k%d" % i, b"v" * i, timestamp=1) for i in range(20)]
    stream, sizes = record.data_table(recs)
    buf = np.frombuffer(stream, np.uint8).copy()
    last = int(sizes[:-1].sum())
    buf[last + 14:last + 22] = np.frombuffer(np.uint64(1 << 40).tobytes(), np.uint8)
    with pytest.raises(_lib.NkvError):
        sstable.make_filter_from_records(buf, sizes, seed=1, ctx=ctx)


def test_bloom_sstable_shape_1m_keys(nkv, oracle):
    """makeFilter at SSTable scale: 1 Mi 16-byte keys at p = 0.01 (M = 10,050,663,
    K = 7), device bits == oracle bits."""
    torch = _torch()
    _lib, ctx = nkv
    ctx.set_stream(torch.cuda.current_stream().cuda_stream)
    L = _lib.lib()
    n = 1 << 20
    data = oracle.splitmix64_bytes(n * 16, 0x6E616B65)
    off = np.arange(n, dtype=np.uint64) * 16
    ln = np.full(n, 16, np.uint64)
    m, k = oracle.bloom_params(n, 0.01)
    d_bits = torch.zeros(((m + 31) // 32) * 4, dtype=torch.uint8, device="cuda")
    d_data, d_off, d_len = _dev(torch, data), _dev(torch, off), _dev(torch, ln)  # held until the kernel ran
    _lib.check(L.nkv_bloom_insert_dev(ctx.h, d_data.data_ptr(), d_off.data_ptr(), d_len.data_ptr(), n,
                                      m, k, 0xABCD1234, d_bits.data_ptr()))
    torch.cuda.synchronize()
    want = oracle.bloom_insert(data, off, ln, m, k, 0xABCD1234)
    assert np.array_equal(d_bits.cpu().numpy()[:want.size], want)


@pytest.mark.parametrize("path", [0, 1, 2])
@pytest.mark.parametrize("n,m,k", [(5000, 47924, 7), (4096, 1, 1), (20000, 5000, 20), (70000, 1 << 22, 3),
                                   (9000, 134217728, 2), (40000, 383416, 40)])
def test_bloom_insert_paths_match_oracle(nkv, oracle, path, n, m, k):
    """Every insert path -- range-privatised (32768-bit ranges in LDS, counting
    sort of the updates), the staged form of it (one hash pass, tiles sorted in
    LDS; k = 40 falls back to the range path) and one atomicOr per bit -- on
    filters of 1 bit to 4096 ranges, k up to 40 (several register passes),
    ragged keys, bits OR-ed into a non-empty filter."""
    torch = _torch()
    _lib, _ = nkv
    ctx = _lib.Context(0)
    ctx.set_stream(torch.cuda.current_stream().cuda_stream)
    ctx.set_option(_lib.NKV_OPT_BLOOM_PATH, path)
    L = _lib.lib()
    rng = np.random.default_rng(n + m + k)
    data, off, ln = _keys(rng, n)
    seed0 = int(rng.integers(0, 2**32))
    words = ((m + 31) // 32) * 4
    pre = np.zeros(words, np.uint8)
    pre[: (m + 7) // 8] = rng.integers(0, 256, (m + 7) // 8, dtype=np.uint8) & rng.integers(0, 2, (m + 7) // 8,
                                                                                          dtype=np.uint8)
    if m % 8:
        pre[(m + 7) // 8 - 1] &= (1 << (m % 8)) - 1
    d_bits = _dev(torch, pre)
    d_data, d_off, d_len = _dev(torch, data), _dev(torch, off), _dev(torch, ln)
    try:
        _lib.check(L.nkv_bloom_insert_dev(ctx.h, d_data.data_ptr(), d_off.data_ptr(), d_len.data_ptr(), n, m, k,
                                          seed0, d_bits.data_ptr()))
        torch.cuda.synchronize()
    finally:
        ctx.close()
    got = d_bits.cpu().numpy()
    want = oracle.bloom_insert(data, off, ln, m, k, seed0) | pre[: (m + 7) // 8]
    assert np.array_equal(got[:want.size], want)
    assert not got[want.size:].any()


@pytest.mark.parametrize("path", [1, 2])
def test_bloom_from_records_range_path(nkv, oracle, path):
    """The records form (keys at rec + 30) through the range-privatised path
    and its staged form."""
    from nakevaleng_amd import record, sstable
    _lib, ctx = nkv
    ctx.set_option(_lib.NKV_OPT_BLOOM_PATH, path)
    rng = np.random.default_rng(44)
    recs = [record.New(rng.integers(0, 256, int(kk), dtype=np.uint8).tobytes(), b"v" * int(v), timestamp=1)
            for kk, v in zip(rng.integers(1, 40, 6000), rng.integers(0, 50, 6000))]
    stream, sizes = record.data_table(recs)
    bf = sstable.make_filter_from_records(stream, sizes, seed=99, ctx=ctx)
    keys = [r.Key for r in recs]
    kd = np.frombuffer(b"".join(keys), np.uint8)
    kl = np.array([len(x) for x in keys], np.uint64)
    ko = np.zeros_like(kl)
    ko[1:] = np.cumsum(kl[:-1])
    ctx.set_option(_lib.NKV_OPT_BLOOM_PATH, 1)
    assert bf.Contents == oracle.bloom_insert(kd, ko, kl, bf.M, bf.K, 99).tobytes()
