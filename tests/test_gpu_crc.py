"""GPU: record checksums -- CRC-32/IEEE of Key || Value
(record.go:51, :163-169) through the C-ABI, against the C oracle (pinned by
the published check value and zlib in test_oracle.py)."""
import ctypes
import zlib

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


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
    return recs, np.frombuffer(stream, np.uint8).copy(), sizes, off


@pytest.mark.parametrize("load", [0, 8])
def test_crc32_spans_every_alignment_and_length(nkv, oracle, load):
    torch = _torch()
    _lib, ctx = nkv
    ctx.set_option(_lib.NKV_OPT_CRC_LOAD, load)
    ctx.set_stream(torch.cuda.current_stream().cuda_stream)
    L = _lib.lib()
    rng = np.random.default_rng(21)
    lens = np.concatenate([np.arange(0, 300), rng.integers(0, 70000, 200), [65536, 65535, 1]]).astype(np.uint64)
    n = lens.size
    off = np.zeros(n, np.uint64)
    off[1:] = np.cumsum(lens[:-1] + rng.integers(0, 16, n - 1).astype(np.uint64))
    data = oracle.splitmix64_bytes(int(off[-1] + lens[-1]) + 1, 99)
    d_data, d_off, d_len = _dev(torch, data), _dev(torch, off), _dev(torch, lens)
    d_out = torch.zeros(n * 4, dtype=torch.uint8, device="cuda")
    _lib.check(L.nkv_crc32_dev(ctx.h, d_data.data_ptr(), d_off.data_ptr(), d_len.data_ptr(), n, d_out.data_ptr()))
    torch.cuda.synchronize()
    got = d_out.cpu().numpy().view(np.uint32)
    want = [oracle.crc32(data[int(o):int(o + l)]) for o, l in zip(off, lens)]
    ctx.set_option(_lib.NKV_OPT_CRC_LOAD, 0)
    assert got.tolist() == want


def test_crc32_check_value(nkv):
    torch = _torch()
    _lib, ctx = nkv
    ctx.set_stream(torch.cuda.current_stream().cuda_stream)
    d = _dev(torch, np.frombuffer(b"123456789", np.uint8))
    o = _dev(torch, np.zeros(1, np.uint64))
    ln = _dev(torch, np.full(1, 9, np.uint64))
    out = torch.zeros(4, dtype=torch.uint8, device="cuda")
    _lib.check(_lib.lib().nkv_crc32_dev(ctx.h, d.data_ptr(), o.data_ptr(), ln.data_ptr(), 1, out.data_ptr()))
    torch.cuda.synchronize()
    assert int(out.cpu().numpy().view(np.uint32)[0]) == 0xCBF43926


@pytest.mark.parametrize("load", [0, 8])
@pytest.mark.parametrize("n", [1, 2, 63, 64, 65, 257, 3000])
def test_record_crc_device_matches_oracle_and_stored(nkv, oracle, n, load):
    torch = _torch()
    _lib, ctx = nkv
    ctx.set_option(_lib.NKV_OPT_CRC_LOAD, load)
    ctx.set_stream(torch.cuda.current_stream().cuda_stream)
    L = _lib.lib()
    rng = np.random.default_rng(n)
    recs, buf, sizes, off = _stream(rng, n)
    bad_idx = sorted(set(rng.integers(0, n, max(1, n // 100)).tolist())) if n > 1 else []
    for i in bad_idx:  # flip one byte of key ++ value (or the stored Crc when empty)
        span = recs[i].KeySize + recs[i].ValueSize
        pos = int(off[i]) + (30 + int(rng.integers(0, span)) if span else 0)
        buf[pos] ^= 0x40
    want_crc, want_ok, want_bad = oracle.record_crcs(buf, off)
    d_buf, d_off = _dev(torch, buf), _dev(torch, off)
    d_crc = torch.zeros(n * 4, dtype=torch.uint8, device="cuda")
    d_stats = torch.zeros(24, dtype=torch.uint8, device="cuda")
    _lib.check(L.nkv_record_crc_dev(ctx.h, d_buf.data_ptr(), buf.size, d_off.data_ptr(), n, d_crc.data_ptr(),
                                    d_stats.data_ptr()))
    torch.cuda.synchronize()
    assert np.array_equal(d_crc.cpu().numpy().view(np.uint32), want_crc)
    stats = d_stats.cpu().numpy().view(np.uint64)
    assert int(stats[0]) == want_bad == len(bad_idx)
    assert int(stats[1]) == (bad_idx[0] if bad_idx else 2**64 - 1)
    assert int(stats[2]) == 0
    ctx.set_option(_lib.NKV_OPT_CRC_LOAD, 0)


def test_record_crc_host_api_and_mirror(nkv, oracle):
    from nakevaleng_amd import record
    _lib, ctx = nkv
    rng = np.random.default_rng(5)
    recs, buf, sizes, off = _stream(rng, 500, vmax=9000)
    crc = record.verify(buf, sizes, ctx)
    assert [int(c) for c in crc] == [r.Crc for r in recs]
    buf[int(off[123]) + 30] ^= 1
    buf[int(off[400]) + 30] ^= 1
    crc2, bad, first = record.checksums(buf, sizes, ctx)
    assert (bad, first) == (2, 123)
    assert int(crc2[123]) == zlib.crc32(buf[int(off[123]) + 30:int(off[123] + sizes[123])].tobytes())
    with pytest.raises(ValueError, match="^Bad Record checksum"):
        record.verify(buf, sizes, ctx)


def test_record_crc_header_outside_stream(nkv):
    torch = _torch()
    _lib, ctx = nkv
    from nakevaleng_amd import record
    rng = np.random.default_rng(6)
    recs, buf, sizes, off = _stream(rng, 10)
    buf[int(off[9]) + 22:int(off[9]) + 30] = np.frombuffer(np.uint64(1 << 40).tobytes(), np.uint8)
    with pytest.raises(_lib.NkvError):
        record.checksums(buf, sizes, ctx)


def test_record_crc_sstable_shape_large(nkv, oracle):
    """SSTable records of TotalSize 4096 (16-B key, 4050-B value; SURVEY 8d cfg2
    variant) at 64 Ki records = 256 MiB, device vs oracle, every record."""
    torch = _torch()
    _lib, ctx = nkv
    ctx.set_stream(torch.cuda.current_stream().cuda_stream)
    L = _lib.lib()
    n, ks, vs = 1 << 16, 16, 4050
    body = oracle.splitmix64_bytes(n * 4096, 0x6E616B65).reshape(n, 4096)
    hdr = np.zeros((n, 30), np.uint8)
    hdr[:, 14:22] = np.frombuffer(np.uint64(ks).tobytes(), np.uint8)
    hdr[:, 22:30] = np.frombuffer(np.uint64(vs).tobytes(), np.uint8)
    body[:, :30] = hdr
    off = np.arange(n, dtype=np.uint64) * 4096
    crc, _, _ = oracle.record_crcs(body.reshape(-1), off)
    body[:, 0:4] = crc.view(np.uint8).reshape(n, 4)  # store the right checksums
    d_buf, d_off = _dev(torch, body.reshape(-1)), _dev(torch, off)
    d_crc = torch.zeros(n * 4, dtype=torch.uint8, device="cuda")
    d_stats = torch.zeros(24, dtype=torch.uint8, device="cuda")
    _lib.check(L.nkv_record_crc_dev(ctx.h, d_buf.data_ptr(), body.size, d_off.data_ptr(), n, d_crc.data_ptr(),
                                    d_stats.data_ptr()))
    torch.cuda.synchronize()
    assert np.array_equal(d_crc.cpu().numpy().view(np.uint32), crc)
    assert d_stats.cpu().numpy().view(np.uint64).tolist() == [0, 2**64 - 1, 0]
