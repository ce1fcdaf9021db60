#!/usr/bin/env python3
"""Diagnostic timeline of the fused leaf kernel (stamp build, never the product).

Builds nothing; expects nakevaleng_amd/libnkvmerkle_diag.so (build.py --diag).
Per wave: start / leaf-phase end / end (s_memrealtime, 100 MHz) and s_memtime
(shader clock).  Prints the in-kernel clock, phase shares, and how many waves
are resident over time (tail effect).
"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ["NKV_LIB"] = os.path.join(ROOT, "nakevaleng_amd", "libnkvmerkle_diag.so")

import numpy as np  # noqa: E402
import torch  # noqa: E402

from nakevaleng_amd import _lib  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 20
    vlen = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
    stride = int(sys.argv[3]) if len(sys.argv) > 3 else vlen
    L = _lib.lib()
    L.nkv_diag_set_buffer.argtypes = [ctypes.c_void_p]
    ctx = _lib.Context(0)
    s = torch.cuda.current_stream()
    ctx.set_stream(s.cuda_stream)
    ctx.set_option(_lib.NKV_OPT_LEAF_LOAD, int(os.environ.get("NKV_LEAF_LOAD", "1")))
    mixed = os.environ.get("MIXED") == "1"
    if mixed:
        import bench
        lens_h, off_h = bench.mixed_lengths(4 << 30, bench.SEED_MIXED)
        n = len(lens_h)
        nbytes = int(lens_h.sum())
        d_off = torch.from_numpy(off_h.view(np.int64)).cuda()
        d_len = torch.from_numpy(lens_h.view(np.int64)).cuda()
    else:
        nbytes = n * vlen
    data = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    _lib.check(L.nkv_fill_splitmix64_dev(ctx.h, data.data_ptr(), nbytes, 1))
    nodes = torch.empty(L.nkv_total_nodes(n) * 20, dtype=torch.uint8, device="cuda")
    waves = (n + 255) // 256 * 4
    diag = torch.zeros(waves * 8, dtype=torch.int64, device="cuda")

    def run():
        if mixed:
            _lib.check(L.nkv_tree_from_values_dev(ctx.h, data.data_ptr(), d_off.data_ptr(), d_len.data_ptr(),
                                                  n, nodes.data_ptr()))
        else:
            _lib.check(L.nkv_tree_from_strided_dev(ctx.h, data.data_ptr(), stride, vlen, n, nodes.data_ptr()))
    for _ in range(10):
        run()
    torch.cuda.synchronize()
    assert L.nkv_diag_set_buffer(diag.data_ptr()) == 0
    run()
    torch.cuda.synchronize()
    assert L.nkv_diag_set_buffer(None) == 0
    d = diag.cpu().numpy().view(np.uint64).reshape(waves, 8).astype(np.float64)
    r0, c0, r1, c1, r2, c2 = (d[:, i] for i in range(6))
    t0 = r0.min()
    span_us = (r2.max() - t0) / 100.0
    leaf_us = (r1 - r0) / 100.0
    epi_us = (r2 - r1) / 100.0
    clk = (c2 - c0) / ((r2 - r0) / 100e6) / 1e9
    print(f"n={n} vlen={vlen} waves={waves}  kernel span {span_us:.1f} us")
    print(f"in-kernel clock GHz: median {np.median(clk):.3f}  p5 {np.percentile(clk, 5):.3f}  p95 {np.percentile(clk, 95):.3f}")
    print(f"leaf phase per wave us: median {np.median(leaf_us):.1f} min {leaf_us.min():.1f} max {leaf_us.max():.1f}")
    print(f"fused epilogue per wave us: median {np.median(epi_us):.1f} max {epi_us.max():.1f}")
    starts = (r0 - t0) / 100.0
    ends = (r2 - t0) / 100.0
    grid = np.linspace(0, span_us, 41)
    act = [int(((starts <= x) & (ends > x)).sum()) for x in grid]
    print("resident waves over time (us: waves):")
    print("  " + "  ".join(f"{x:.0f}:{a}" for x, a in zip(grid[::2], act[::2])))
    # waves that start after the first finishes = second round
    first_end = ends.min()
    late = starts > first_end
    print(f"first wave ends at {first_end:.1f} us; {late.sum()} waves start after that; "
          f"last start {starts.max():.1f} us; last end {ends.max():.1f} us")
    xcc = (d[:, 6].astype(np.uint64) >> np.uint64(32)).astype(int)
    dur = ends - starts
    order = np.argsort(-dur)
    print("longest waves (us): " + ", ".join(f"w{int(i)} start {starts[i]:.0f} dur {dur[i]:.0f}" for i in order[:6]))
    hw = (d[:, 6].astype(np.uint64) & np.uint64(0xFFFFFFFF)).astype(np.int64)
    xcc_all = (d[:, 6].astype(np.uint64) >> np.uint64(32)).astype(np.int64)
    simd = (hw >> 4) & 3
    cu = (hw >> 8) & 15
    sh = (hw >> 12) & 1
    se = (hw >> 13) & 7
    simd_key = (((xcc_all * 8 + se) * 2 + sh) * 16 + cu) * 4 + simd
    cu_key = simd_key // 4
    top = order[:1024]
    from collections import Counter
    cs = Counter(simd_key[top].tolist())
    cc = Counter(cu_key[top].tolist())
    print(f"1024 longest waves: on {len(cs)} distinct SIMDs (max {max(cs.values())} per SIMD), "
          f"{len(cc)} distinct CUs (max {max(cc.values())} per CU); all waves on {len(set(simd_key.tolist()))} SIMDs")
    wpsimd = Counter(simd_key.tolist())
    print(f"waves per SIMD over the kernel: min {min(wpsimd.values())} max {max(wpsimd.values())}")
    for x in range(8):
        m = xcc == x
        if m.any():
            print(f"  xcc {x}: waves {m.sum()}  last end {ends[m].max():.1f} us  median leaf {np.median(leaf_us[m]):.1f}")
    ctx.close()


if __name__ == "__main__":
    main()
