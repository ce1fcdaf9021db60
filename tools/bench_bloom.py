#!/usr/bin/env python3
"""SSTable filter build throughput: makeFilter's murmur3
Bloom inserts (sstable.go:49-56) for 1 Mi records of TotalSize 4096 whose
16-byte keys sit in a device-resident Data table (key at rec + 30), p = 0.01
(M = 10,050,663 bits, K = 7).  HIP events on the library's stream; prints one
JSON line with keys/s, the kernel time, and the C oracle on one core."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from nakevaleng_amd import _lib, bloomfilter  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--records", type=int, default=1 << 20)
    ap.add_argument("--rec-bytes", type=int, default=4096)
    ap.add_argument("--key-bytes", type=int, default=16)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--verify", action="store_true")
    ap.add_argument("--path", type=int, default=-1, help="NKV_OPT_BLOOM_PATH override")
    args = ap.parse_args()
    n, rb, ks = args.records, args.rec_bytes, args.key_bytes
    L = _lib.lib()
    ctx = _lib.Context(0)
    s = torch.cuda.current_stream()
    ctx.set_stream(s.cuda_stream)
    if args.path >= 0:
        ctx.set_option(_lib.NKV_OPT_BLOOM_PATH, args.path)
    m, k = bloomfilter.params(n, 0.01)
    seed0 = 0x6E616B65
    data = torch.empty(n * rb, dtype=torch.uint8, device="cuda")
    _lib.check(L.nkv_fill_splitmix64_dev(ctx.h, data.data_ptr(), n * rb, seed0))
    off = torch.arange(n, dtype=torch.int64, device="cuda") * rb + 30
    ln = torch.full((n,), ks, dtype=torch.int64, device="cuda")
    bits = torch.zeros(((m + 31) // 32) * 4, dtype=torch.uint8, device="cuda")

    def run():
        _lib.check(L.nkv_bloom_insert_dev(ctx.h, data.data_ptr(), off.data_ptr(), ln.data_ptr(), n, m, k, seed0,
                                          bits.data_ptr()))
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
    out = {"metric": "SSTable filter build (murmur3 Bloom inserts), keys/s", "value": round(n / (ms * 1e-3), 1),
           "unit": "keys/s", "ms_per_launch": round(ms, 4), "keys": n, "key_bytes": ks, "m_bits": m, "k": k,
           "bit_updates_per_s": round(n * k / (ms * 1e-3), 1)}
    from oracle import oracle_c as oc  # CPU baseline / checker only
    sample = 1 << 16
    hd = data.view(n, rb)[:sample, 30:30 + ks].cpu().numpy().reshape(-1).copy()
    hoff = np.arange(sample, dtype=np.uint64) * ks
    hln = np.full(sample, ks, np.uint64)
    t0 = time.perf_counter()
    oc.bloom_insert(hd, hoff, hln, m, k, seed0)
    dt = time.perf_counter() - t0
    out["cpu_baseline"] = {"value": round(sample / dt, 1), "unit": "keys/s", "cores": 1, "kind": "port",
                           "sample": f"first {sample} keys, C oracle"}
    if args.verify:
        hk = data.view(n, rb)[:, 30:30 + ks].cpu().numpy().reshape(-1).copy()
        want = oc.bloom_insert(hk, np.arange(n, dtype=np.uint64) * ks, np.full(n, ks, np.uint64), m, k, seed0)
        out["verified_vs_oracle"] = bool(np.array_equal(bits.cpu().numpy()[:want.size], want))
    print(json.dumps(out), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
