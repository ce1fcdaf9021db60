#!/usr/bin/env python3
"""Diagnostic timeline of the work-queue leaf kernel on the mixed config
(stamp build libnkvmerkle_diag.so, never the product).

Per wave: start/end (s_memrealtime, 100 MHz), shader clocks, SIMD key and
arrival slot, groups pulled, and the sum over those groups of the longest chain
in 64-B blocks.  Prints how the front (slot 0) and back waves spent the kernel.
"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ["NKV_LIB"] = os.path.join(ROOT, "nakevaleng_amd", "libnkvmerkle_diag.so")

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from nakevaleng_amd import _lib  # noqa: E402


def main():
    L = _lib.lib()
    L.nkv_diag_set_buffer.argtypes = [ctypes.c_void_p]
    ctx = _lib.Context(0)
    ctx.set_stream(torch.cuda.current_stream().cuda_stream)
    deep = int(os.environ.get("DEEP", "3"))
    qwaves = int(os.environ.get("QWAVES", "4"))
    ctx.set_option(_lib.NKV_OPT_QUEUE_WAVES, qwaves)
    ctx.set_option(_lib.NKV_OPT_QUEUE_SPLIT, int(os.environ.get("QSPLIT", "32")))
    ring = int(os.environ.get("RING", "13"))
    ctx.set_option(_lib.NKV_OPT_BUCKET, 1)
    lens_h, off_h = bench.mixed_lengths(4 << 30, bench.SEED_MIXED)
    n = len(lens_h)
    nbytes = int(lens_h.sum())
    d_off = torch.from_numpy(off_h.view(np.int64)).cuda()
    d_len = torch.from_numpy(lens_h.view(np.int64)).cuda()
    data = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    _lib.check(L.nkv_fill_splitmix64_dev(ctx.h, data.data_ptr(), nbytes, 1))
    nodes = torch.empty(L.nkv_total_nodes(n) * 20, dtype=torch.uint8, device="cuda")
    simds = torch.cuda.get_device_properties(0).multi_processor_count * 4
    slots = ring % 10
    waves = (min(qwaves, 2 if slots == 4 else (3 if slots == 3 else 5)) if deep == 3 else 2) * simds
    diag = torch.zeros(waves * 8, dtype=torch.int64, device="cuda")

    def run():
        _lib.check(L.nkv_tree_from_values_dev(ctx.h, data.data_ptr(), d_off.data_ptr(), d_len.data_ptr(),
                                              n, nodes.data_ptr()))
    for _ in range(10):
        run()
    torch.cuda.synchronize()
    assert L.nkv_diag_set_buffer(diag.data_ptr()) == 0
    run()
    torch.cuda.synchronize()
    assert L.nkv_diag_set_buffer(None) == 0
    d = diag.cpu().numpy().view(np.uint64).reshape(waves, 8)
    r0, r1, c0, c1 = (d[:, i].astype(np.float64) for i in range(4))
    key = (d[:, 4] & 0xFFFFFFFF).astype(np.int64)
    slot = (d[:, 4] >> 32).astype(np.int64)
    groups, blocks, first = d[:, 5].astype(np.int64), d[:, 6].astype(np.int64), d[:, 7].astype(np.float64)
    t0 = r0.min()
    span = (r1.max() - t0) / 100.0
    clk = (c1 - c0) / ((r1 - r0) / 100e6) / 1e9
    print(f"n={n} groups={(n + 63) // 64} waves={waves} kernel span {span:.1f} us, clock median {np.median(clk):.3f} GHz")
    print(f"distinct SIMD keys {len(np.unique(key))}; slot histogram {np.bincount(slot).tolist()}")
    per_simd = np.bincount(np.unique(key, return_inverse=True)[1])
    print(f"waves per SIMD: {np.bincount(per_simd).tolist()} (index = waves)")
    print(f"groups pulled: total {groups.sum()}; blocks sum {blocks.sum()}")
    for name, m in (("front", slot == 0), ("back", slot != 0)):
        st = (r0[m] - t0) / 100.0
        en = (r1[m] - t0) / 100.0
        fe = (first[m] - t0) / 100.0
        print(f"{name}: {m.sum()} waves; start us p50 {np.median(st):.1f} max {st.max():.1f}; "
              f"first group done p50 {np.median(fe):.1f} max {fe.max():.1f}; end p50 {np.median(en):.1f} "
              f"min {en.min():.1f} max {en.max():.1f}; groups/wave p50 {np.median(groups[m]):.0f} max {groups[m].max()}; "
              f"blocks/wave p50 {np.median(blocks[m]):.0f} max {blocks[m].max()}")
    # per-SIMD total blocks (all its waves) vs its end time
    inv = np.unique(key, return_inverse=True)[1]
    sb = np.bincount(inv, weights=blocks)
    se = np.zeros(len(sb))
    np.maximum.at(se, inv, (r1 - t0) / 100.0)
    print(f"per-SIMD blocks: min {sb.min():.0f} p50 {np.median(sb):.0f} max {sb.max():.0f}; "
          f"per-SIMD end us: min {se.min():.1f} p50 {np.median(se):.1f} max {se.max():.1f}")
    worst = np.argsort(-se)[:5]
    for w in worst:
        ws = np.where(inv == w)[0]
        print(f"  slow SIMD key {np.unique(key)[w]}: end {se[w]:.1f} us, blocks {sb[w]:.0f}, waves "
              + ", ".join(f"[slot {slot[i]} g {groups[i]} b {blocks[i]} {((r0[i]-t0)/100):.0f}-{((r1[i]-t0)/100):.0f}]" for i in ws))
    print(f"us per block on a front wave's first group: "
          f"{np.median(((first - r0) / 100.0)[slot == 0]):.1f} us total")


if __name__ == "__main__":
    main()
