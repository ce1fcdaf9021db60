#!/usr/bin/env python3
"""A/B experiments on the leaf kernel, interleaved rounds in one process.

Each variant times nkv_tree_from_strided_dev (or the non-fused leaf kernel)
with HIP events on the library's stream; prints median/min GB/s of payload.
"""
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from nakevaleng_amd import _lib  # noqa: E402


def main():
    L = _lib.lib()
    ctx = _lib.Context(0)
    s = torch.cuda.current_stream()
    ctx.set_stream(s.cuda_stream)
    big = torch.empty(2 * (1 << 20) * 4096, dtype=torch.uint8, device="cuda")
    _lib.check(L.nkv_fill_splitmix64_dev(ctx.h, big.data_ptr(), big.numel(), 1))
    nodes = torch.empty(L.nkv_total_nodes(8 << 20) * 20, dtype=torch.uint8, device="cuda")

    def fused(n, stride, vlen):
        return lambda: L.nkv_tree_from_strided_dev(ctx.h, big.data_ptr(), stride, vlen, n, nodes.data_ptr())

    def leaf_only(n, stride, vlen):
        return lambda: L.nkv_leaf_hash_strided_dev(ctx.h, big.data_ptr(), stride, vlen, n, nodes.data_ptr())

    def with_load(mode, fn):
        def run():
            ctx.set_option(_lib.NKV_OPT_LEAF_LOAD, mode)
            return fn()
        return run

    M = 1 << 20
    variants = {}
    import numpy as np
    sel = os.environ.get("EXP", "loads")
    if sel == "loads":
        for mode, name in ((1, "lds-dma"), (2, "direct"), (4, "runs128"), (5, "runs256")):
            variants[f"{name:10s} fused 1Mx4K"] = (with_load(mode, fused(M, 4096, 4096)), M * 4096)
            variants[f"{name:10s} leafonly 1Mx4K"] = (with_load(mode, leaf_only(M, 4096, 4096)), M * 4096)
            variants[f"{name:10s} fused 1Mx4K stride0"] = (with_load(mode, fused(M, 0, 4096)), M * 4096)
            variants[f"{name:10s} fused 4Mx1K"] = (with_load(mode, fused(4 * M, 1024, 1024)), 4 * M * 1024)
    elif sel == "long":
        # few, long chains: 1 and 2 waves per SIMD
        for mode, name in ((1, "lds-dma"), (2, "direct"), (5, "runs256")):
            variants[f"{name:8s} 64K x 64KiB (1 wave/SIMD)"] = (with_load(mode, fused(65536, 65536, 65536)), 65536 * 65536)
            variants[f"{name:8s} 128K x 32KiB (2 waves/SIMD)"] = (with_load(mode, fused(131072, 32768, 32768)), 131072 * 32768)
        offl = torch.from_numpy(np.arange(65536, dtype=np.int64) * 65536).cuda()
        lenl = torch.full((65536,), 65536, dtype=torch.int64, device="cuda")
        for deep in (0, 1):
            def runl(deep=deep):
                ctx.set_option(_lib.NKV_OPT_DEEP_PREFETCH, deep)
                return L.nkv_tree_from_values_dev(ctx.h, big.data_ptr(), offl.data_ptr(), lenl.data_ptr(), 65536,
                                                  nodes.data_ptr())
            variants[f"offsets bucketed deep={deep} 64K x 64KiB"] = (runl, 65536 * 65536)
    else:
        # funnel (unaligned) vs aligned, strided and offset-array paths
        variants["strided aligned 1Mx4096"] = (fused(M, 4096, 4096), M * 4096)
        base46 = big.data_ptr() + 46
        variants["strided unaligned(+46) 1Mx4050"] = (
            lambda: L.nkv_tree_from_strided_dev(ctx.h, base46, 4096, 4050, M, nodes.data_ptr()), M * 4050)
        off_a = torch.from_numpy((np.arange(M, dtype=np.int64) * 4096)).cuda()
        off_u = torch.from_numpy((np.arange(M, dtype=np.int64) * 4096 + 46)).cuda()
        len_a = torch.full((M,), 4096, dtype=torch.int64, device="cuda")
        len_u = torch.full((M,), 4050, dtype=torch.int64, device="cuda")

        def offs(o, l, bucket):
            def run():
                ctx.set_option(_lib.NKV_OPT_BUCKET, bucket)
                return L.nkv_tree_from_values_dev(ctx.h, big.data_ptr(), o.data_ptr(), l.data_ptr(), M,
                                                  nodes.data_ptr())
            return run
        variants["offsets aligned bucket0"] = (offs(off_a, len_a, 0), M * 4096)
        variants["offsets aligned bucket1"] = (offs(off_a, len_a, 1), M * 4096)
        variants["offsets unaligned bucket0"] = (offs(off_u, len_u, 0), M * 4050)
        variants["offsets unaligned bucket1"] = (offs(off_u, len_u, 1), M * 4050)
    res = {k: [] for k in variants}
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    for fn, _ in variants.values():
        _lib.check(fn())
    torch.cuda.synchronize()
    for _ in range(int(os.environ.get("ROUNDS", "5"))):
        for k, (fn, nbytes) in variants.items():
            e0.record(s)
            for _ in range(3):
                _lib.check(fn())
            e1.record(s)
            e1.synchronize()
            ms = e0.elapsed_time(e1) / 3
            res[k].append(nbytes / (ms * 1e-3) / 1e9)
    for k, v in res.items():
        print(f"{k:40s} median {statistics.median(v):8.1f} GB/s  max {max(v):8.1f}")
    ctx.close()


if __name__ == "__main__":
    main()
