#!/usr/bin/env python3
"""Where the one-launch small tree's time goes (stamp build, never the product).

Expects nakevaleng_amd/libnkvmerkle_diag.so (build.py --diag).  Calls
nkv_tree_from_values on the reference's default flush (10 values of 1..200
bytes, tools/small_flush.cpp's generator) REPS times back to back, the stamps
of the last call kept: per wave, s_memrealtime (100 MHz) and s_memtime (shader
clock) at kernel entry, after the input staging, after the leaf hashes and
after the tree levels.  Prints the phase durations (us) and the shader clock
each phase ran at, median over the waves of K sampled calls.

    python tools/small_diag.py [N [MINLEN MAXLEN [REPS [K]]]]
"""
import ctypes
import json
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
    a = sys.argv[1:]
    n = int(a[0]) if a else 10
    lo, hi = (int(a[1]), int(a[2])) if len(a) > 2 else (1, 200)
    reps = int(a[3]) if len(a) > 3 else 200
    k = int(a[4]) if len(a) > 4 else 50
    L = _lib.lib()
    L.nkv_diag_set_buffer.argtypes = [ctypes.c_void_p]
    ctx = _lib.Context(0)
    data, off, ln = bench.small_shape_values(n, lo, hi)
    data = np.concatenate([data, np.zeros(16, np.uint8)])
    tot = L.nkv_total_nodes(n)
    root = np.zeros(20, np.uint8)
    nodes = np.zeros(20 * tot, np.uint8)
    img = np.zeros(L.nkv_bfs_size(n), np.uint8)
    waves = (n + 255) // 256 * 4
    diag = torch.zeros(waves * 8, dtype=torch.int64, device="cuda")

    def call():
        _lib.check(L.nkv_tree_from_values(ctx.h, _lib.p8(data), _lib.p64(off), _lib.p64(ln), n, _lib.p8(root),
                                          _lib.p8(nodes), _lib.p8(img)))
    for _ in range(reps):
        call()
    rows = []
    for _ in range(k):
        diag.zero_()
        torch.cuda.synchronize()
        assert L.nkv_diag_set_buffer(diag.data_ptr()) == 0
        call()
        torch.cuda.synchronize()
        assert L.nkv_diag_set_buffer(None) == 0
        d = diag.cpu().numpy().view(np.uint64).reshape(waves, 8).astype(np.float64)
        live = d[:, 0] > 0
        rows.append(d[live])
    d = np.concatenate(rows)
    r = [d[:, 2 * j] for j in range(4)]
    c = [d[:, 2 * j + 1] for j in range(4)]
    out = {"n": n, "value_bytes": [lo, hi], "calls_sampled": k, "waves": int(d.shape[0]), "path": ctx.last_path()}
    for name, j0, j1 in (("stage_in", 0, 1), ("leaves", 1, 2), ("tree", 2, 3)):
        m = r[j1] > 0
        us = (r[j1][m] - r[j0][m]) / 100.0
        ghz = (c[j1][m] - c[j0][m]) / np.maximum(r[j1][m] - r[j0][m], 1) * 100e6 / 1e9
        out[name] = {"us_median": round(float(np.median(us)), 2), "us_p90": round(float(np.percentile(us, 90)), 2),
                     "ghz_median": round(float(np.median(ghz)), 3)}
    print(json.dumps(out), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
