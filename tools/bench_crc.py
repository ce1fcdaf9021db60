#!/usr/bin/env python3
"""Record-checksum throughput: CRC-32/IEEE of Key || Value
over a device-resident Data-table stream of SSTable-shaped records (TotalSize
4096: 16-B key, 4050-B value; 1 Mi records = 4 GiB), checked against the
stored Crc of every record (record.Deserialize's check, record.go:163-169).

Prints one JSON line: GB/s of checksummed bytes (Key || Value) per launch from
HIP events on the library's stream, the HBM roofline fraction, and the C
oracle's single-thread rate on a bounded sample.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from nakevaleng_amd import _lib  # noqa: E402

HBM_PEAK_GBS = 8000.0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--records", type=int, default=1 << 20)
    ap.add_argument("--rec-bytes", type=int, default=4096)
    ap.add_argument("--key-bytes", type=int, default=16)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--verify", action="store_true")
    ap.add_argument("--crc-load", type=int, default=-1, help="NKV_OPT_CRC_LOAD override")
    args = ap.parse_args()
    n, rb, ks = args.records, args.rec_bytes, args.key_bytes
    vs = rb - 30 - ks
    L = _lib.lib()
    ctx = _lib.Context(0)
    s = torch.cuda.current_stream()
    ctx.set_stream(s.cuda_stream)
    if args.crc_load >= 0:
        ctx.set_option(_lib.NKV_OPT_CRC_LOAD, args.crc_load)
    data = torch.empty(n * rb, dtype=torch.uint8, device="cuda")
    _lib.check(L.nkv_fill_splitmix64_dev(ctx.h, data.data_ptr(), n * rb, 0x6E616B65))
    v = data.view(n, rb)
    v[:, 14:22] = torch.from_numpy(np.frombuffer(np.uint64(ks).tobytes(), np.uint8).copy()).cuda()
    v[:, 22:30] = torch.from_numpy(np.frombuffer(np.uint64(vs).tobytes(), np.uint8).copy()).cuda()
    off = torch.arange(n, dtype=torch.int64, device="cuda") * rb
    crc = torch.empty(n * 4, dtype=torch.uint8, device="cuda")
    stats = torch.empty(24, dtype=torch.uint8, device="cuda")

    def run():
        _lib.check(L.nkv_record_crc_dev(ctx.h, data.data_ptr(), n * rb, off.data_ptr(), n, crc.data_ptr(),
                                        stats.data_ptr()))
    run()
    torch.cuda.synchronize()
    v[:, 0:4] = crc.view(n, 4)  # store the checksums: every record must now verify
    for _ in range(args.warmup):
        run()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(args.steps):
        run()
    e1.record(s)
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / args.steps
    st = stats.cpu().numpy().view(np.uint64).tolist()
    span_bytes = n * (ks + vs)
    gbs = span_bytes / (ms * 1e-3) / 1e9
    out = {"metric": "record CRC-32 (Key || Value) verify, GB/s of checksummed bytes", "value": round(gbs, 1),
           "load": args.crc_load,
           "unit": "GB/s", "ms_per_launch": round(ms, 4), "records": n, "record_bytes": rb,
           "bad_records": st[0], "roofline": {"bound": "hbm", "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS,
                                              "unit": "GB/s", "frac": round(gbs / HBM_PEAK_GBS, 4)}}
    from oracle import oracle_c as oc  # CPU baseline / checker only
    sample = 4096
    host = v[:sample].cpu().numpy().reshape(-1).copy()
    hoff = np.arange(sample, dtype=np.uint64) * rb
    t0 = time.perf_counter()
    hc, ok, bad = oc.record_crcs(host, hoff)
    dt = time.perf_counter() - t0
    out["cpu_baseline"] = {"value": round(sample * (ks + vs) / dt / 1e9, 3), "unit": "GB/s", "cores": 1,
                           "kind": "port", "sample": f"first {sample} records, bitwise C oracle"}
    if args.verify:
        out["verified_vs_oracle"] = bool(bad == 0 and np.array_equal(hc, crc.view(n, 4)[:sample].cpu().numpy()
                                                                       .reshape(-1).view(np.uint32)))
    print(json.dumps(out), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
