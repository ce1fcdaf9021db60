"""GPU: seeded randomized parity sweep over the C-ABI entry points, batch shapes
and context options together, against the C oracle.

Each case draws one entry point (device offsets, host values, strided, records
on the device or the host, the CRC-verified compaction read), a batch shape
(one length, small ragged, log-uniform 64 B - 64 KiB like configs[2], zeros
mixed in), a layout (packed back to back, so mostly unaligned, or with random
gaps) and a fresh context with random options (load path, ordering policy,
queue waves / split, records plan, table lanes, host staging threads and chunk).
Every combination must give the oracle's tree: the options choose kernels,
never results.  Reference:
merklenode.go:27-34 (leaf), merkletree.go:31-64 (tree), record.go:191-199
(record layout), record.go:163-169 (Crc).
"""
import zlib

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

CASES = 192
MAX_BYTES = 24 << 20  # per case, so the oracle side stays well under a second

ENTRIES = ["values_dev", "values_host", "strided_dev", "records_dev", "records_host", "verify_dev"]


def _options(rng, _lib):
    return {
        _lib.NKV_OPT_LEAF_LOAD: int(rng.choice([4, 11])),
        _lib.NKV_OPT_BUCKET: int(rng.integers(0, 3)),
        _lib.NKV_OPT_QUEUE_WAVES: int(rng.integers(1, 4)),
        _lib.NKV_OPT_TABLE_LANES: int(rng.integers(1, 4)),
        _lib.NKV_OPT_QUEUE_SPLIT: int(rng.choice([0, 1, 8, 32, 1000])),
        _lib.NKV_OPT_RECORDS_FUSED: int(rng.integers(0, 2)),
        _lib.NKV_OPT_HOST_THREADS: int(rng.choice([0, 1, 3, 16])),
        _lib.NKV_OPT_STAGE_CHUNK: int(rng.choice([4096, 65536, 32 << 20])),
        _lib.NKV_OPT_SIDE_GATE: int(rng.integers(0, 2)),
    }


def _lengths(rng, n):
    kind = int(rng.integers(0, 4))
    if kind == 0:  # one size (an SSTable of one record size)
        lens = np.full(n, int(rng.integers(0, 9000)), np.uint64)
    elif kind == 1:  # small and ragged
        lens = rng.integers(0, 200, n).astype(np.uint64)
    elif kind == 2:  # configs[2]: log-uniform 64 B - 64 KiB
        lens = np.floor(2.0 ** rng.uniform(6, 16, n)).astype(np.uint64)
    else:  # mostly one size, some empty, some long
        lens = np.full(n, 4050, np.uint64)
        k = max(1, n // 20)
        lens[rng.integers(0, n, k)] = 0
        lens[rng.integers(0, n, k)] = rng.integers(5000, 40000, k).astype(np.uint64)
    while int(lens.sum()) > MAX_BYTES and n > 1:  # keep the case small
        n //= 2
        lens = lens[:n]
    return lens


def _case(seed):
    rng = np.random.default_rng(0xF022 + seed)
    entry = ENTRIES[seed % len(ENTRIES)]
    n = int(np.exp(rng.uniform(0, np.log(20000))))
    return rng, entry, max(1, n)


@pytest.mark.parametrize("seed", range(CASES))
def test_fuzz_parity(oracle, seed):
    import torch
    from nakevaleng_amd import _lib, record
    L = _lib.lib()
    rng, entry, n = _case(seed)
    ctx = _lib.Context(0)
    try:
        for k, v in _options(rng, _lib).items():
            ctx.set_option(k, v)
        if entry in ("values_dev", "values_host"):
            lens = _lengths(rng, n)
            n = len(lens)
            gaps = rng.integers(0, 100, n).astype(np.uint64) if rng.integers(0, 2) else np.zeros(n, np.uint64)
            off = np.zeros(n, np.uint64)
            if n > 1:
                off[1:] = np.cumsum(lens[:-1] + gaps[:-1])
            total = int(off[-1] + lens[-1]) + 1
            data = oracle.splitmix64_bytes(total, seed)
            want = oracle.tree_from_digests(oracle.leaf_hashes(data, off, lens, threads=8))
            nodes = np.zeros((L.nkv_total_nodes(n), 20), np.uint8)
            if entry == "values_host":
                _lib.check(L.nkv_tree_from_values(ctx.h, _lib.p8(data), _lib.p64(off), _lib.p64(lens), n, None,
                                                  _lib.p8(nodes), None))
            else:
                with ctx.on_stream(torch.cuda.current_stream().cuda_stream):
                    d = torch.from_numpy(data).cuda()
                    d_off = torch.from_numpy(off.view(np.int64)).cuda()
                    d_len = torch.from_numpy(lens.view(np.int64)).cuda()
                    d_nodes = torch.zeros(nodes.size, dtype=torch.uint8, device="cuda")
                    _lib.check(L.nkv_tree_from_values_dev(ctx.h, d.data_ptr(), d_off.data_ptr(), d_len.data_ptr(),
                                                          n, d_nodes.data_ptr()))
                    nodes = d_nodes.cpu().numpy().reshape(-1, 20)
            assert np.array_equal(nodes, want), (entry, n)
        elif entry == "strided_dev":
            vlen = int(rng.integers(0, 9000))
            stride = vlen + int(rng.choice([0, 1, 16, 64, 100]))
            n = max(1, min(n, MAX_BYTES // max(stride, 1)))
            data = oracle.splitmix64_bytes(n * stride + 1, seed)
            want = oracle.tree_from_digests(oracle.leaf_hashes_strided(data, stride, vlen, n, threads=8))
            with ctx.on_stream(torch.cuda.current_stream().cuda_stream):
                d = torch.from_numpy(data).cuda()
                d_nodes = torch.zeros(L.nkv_total_nodes(n) * 20, dtype=torch.uint8, device="cuda")
                _lib.check(L.nkv_tree_from_strided_dev(ctx.h, d.data_ptr(), stride, vlen, n, d_nodes.data_ptr()))
                got = d_nodes.cpu().numpy().reshape(-1, 20)
            assert np.array_equal(got, want), (entry, n, stride, vlen)
        else:  # records
            vl = _lengths(rng, n)
            n = len(vl)
            kls = rng.integers(0, 40, n)
            recs = [record.New(rng.bytes(int(kls[i])), rng.bytes(int(vl[i])), timestamp=i) for i in range(n)]
            stream, sizes = record.data_table(recs)
            buf = np.frombuffer(stream, np.uint8).copy()
            roff = np.zeros(n, np.uint64)
            roff[1:] = np.cumsum(np.asarray(sizes, np.uint64)[:-1])
            off, ln = record.value_spans(stream, sizes)
            want = oracle.tree_from_digests(oracle.leaf_hashes(buf, off, ln, threads=8))
            if entry == "records_host":
                rs = np.ascontiguousarray(sizes, dtype=np.uint64)
                hb = np.frombuffer(stream + b"\0", np.uint8)
                nodes = np.zeros((L.nkv_total_nodes(n), 20), np.uint8)
                _lib.check(L.nkv_tree_from_records(ctx.h, _lib.p8(hb), len(stream), _lib.p64(rs), n, None,
                                                   _lib.p8(nodes), None))
                assert np.array_equal(nodes, want), (entry, n)
                return
            bad = -1
            if entry == "verify_dev" and n > 2 and rng.integers(0, 2):
                bad = int(rng.integers(0, n))
                buf[int(roff[bad])] ^= 0x01  # one stored Crc wrong
            with ctx.on_stream(torch.cuda.current_stream().cuda_stream):
                d = torch.from_numpy(buf).cuda()
                d_roff = torch.from_numpy(roff.view(np.int64)).cuda()
                d_nodes = torch.zeros(L.nkv_total_nodes(n) * 20, dtype=torch.uint8, device="cuda")
                if entry == "records_dev":
                    d_err = torch.full((1,), 3, dtype=torch.int32, device="cuda")
                    _lib.check(L.nkv_tree_from_records_dev(ctx.h, d.data_ptr(), len(stream), d_roff.data_ptr(), n,
                                                           d_nodes.data_ptr(), d_err.data_ptr()))
                    assert int(d_err.item()) == 0
                else:
                    d_crc = torch.zeros(n, dtype=torch.int32, device="cuda")
                    d_stats = torch.zeros(3, dtype=torch.int64, device="cuda")
                    _lib.check(L.nkv_tree_verify_records_dev(ctx.h, d.data_ptr(), len(stream), d_roff.data_ptr(),
                                                             n, d_nodes.data_ptr(), d_crc.data_ptr(),
                                                             d_stats.data_ptr()))
                    crcs = np.array([zlib.crc32(buf[int(roff[i]) + 30:int(off[i] + ln[i])].tobytes())
                                     for i in range(n)], np.uint32)
                    assert np.array_equal(d_crc.cpu().numpy().view(np.uint32), crcs)
                    assert d_stats.cpu().tolist() == ([1, bad, 0] if bad >= 0 else [0, -1, 0])
                got = d_nodes.cpu().numpy().reshape(-1, 20)
            assert np.array_equal(got, want), (entry, n)
    finally:
        ctx.close()


@pytest.mark.parametrize("seed", range(96))
def test_fuzz_crc_bloom(oracle, seed):
    """Span checksums (every NKV_OPT_CRC_LOAD kernel) and filter inserts and
    queries (every NKV_OPT_BLOOM_PATH) over random spans at random alignments,
    random m, k and seeds, against the oracle (record.go:51, bloomfilter.go:76-91)."""
    import torch
    from nakevaleng_amd import _lib
    L = _lib.lib()
    rng = np.random.default_rng(0xC0C + seed)
    n = int(np.exp(rng.uniform(0, np.log(30000))))
    lens = (rng.integers(0, 64, n) if rng.integers(0, 2) else rng.integers(0, 6000, n)).astype(np.uint64)
    gaps = rng.integers(0, 40, n).astype(np.uint64)
    off = np.zeros(n, np.uint64)
    if n > 1:
        off[1:] = np.cumsum(lens[:-1] + gaps[:-1])
    data = oracle.splitmix64_bytes(int(off[-1] + lens[-1]) + 1, seed)
    ctx = _lib.Context(0)
    try:
        ctx.set_option(_lib.NKV_OPT_CRC_LOAD, int(rng.choice([0, 8])))
        ctx.set_option(_lib.NKV_OPT_BLOOM_PATH, int(rng.integers(0, 3)))
        m = int(rng.integers(1, 1 << 21))
        k = int(rng.integers(1, 21))
        seed0 = int(rng.integers(0, 1 << 32))
        with ctx.on_stream(torch.cuda.current_stream().cuda_stream):
            d = torch.from_numpy(data).cuda()
            d_off = torch.from_numpy(off.view(np.int64)).cuda()
            d_len = torch.from_numpy(lens.view(np.int64)).cuda()
            d_crc = torch.zeros(n, dtype=torch.int32, device="cuda")
            _lib.check(L.nkv_crc32_dev(ctx.h, d.data_ptr(), d_off.data_ptr(), d_len.data_ptr(), n, d_crc.data_ptr()))
            d_bits = torch.zeros((m + 31) // 32 * 4, dtype=torch.uint8, device="cuda")  # whole words (header)
            _lib.check(L.nkv_bloom_insert_dev(ctx.h, d.data_ptr(), d_off.data_ptr(), d_len.data_ptr(), n, m, k, seed0,
                                              d_bits.data_ptr()))
            # queries: the inserted keys in reverse order plus keys shifted by one byte
            q_off = np.concatenate([off[::-1], off + 1]).astype(np.uint64)
            q_len = np.concatenate([lens[::-1], lens]).astype(np.uint64)
            d_qoff = torch.from_numpy(q_off.view(np.int64)).cuda()
            d_qlen = torch.from_numpy(q_len.view(np.int64)).cuda()
            d_hit = torch.zeros(2 * n, dtype=torch.uint8, device="cuda")
            _lib.check(L.nkv_bloom_query_dev(ctx.h, d.data_ptr(), d_qoff.data_ptr(), d_qlen.data_ptr(), 2 * n, m, k,
                                             seed0, d_bits.data_ptr(), d_hit.data_ptr()))
            crc = d_crc.cpu().numpy().view(np.uint32)
            bits = d_bits.cpu().numpy()
            hit = d_hit.cpu().numpy()
        want_crc = np.array([oracle.crc32(data[int(off[i]):int(off[i] + lens[i])]) for i in range(n)], np.uint32)
        assert np.array_equal(crc, want_crc)
        want_bits = oracle.bloom_insert(data, off, lens, m, k, seed0)
        assert np.array_equal(bits[:(m + 7) // 8], want_bits)
        assert not bits[(m + 7) // 8:].any()  # the word padding stays zero
        want_hit = oracle.bloom_query(data, q_off, q_len, m, k, seed0, want_bits)
        assert np.array_equal(hit.astype(bool), want_hit[:2 * n].astype(bool))
        assert hit[:n].all()  # no false negatives
    finally:
        ctx.close()
