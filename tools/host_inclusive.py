#!/usr/bin/env python3
"""Host-inclusive rate of the Merkle step (DESIGN.md "Host-inclusive rate").

The path starts and ends in host memory: memtable values on flush, Data-table
bytes on compaction; the metadata image goes back to the host to be written.
Two measurements on BASELINE configs[1] (1 Mi x 4 KiB):
  (a) nkv_tree_from_values, the synchronous host API: a pool of host threads
      gathers values into pinned staging chunks while earlier chunks are in
      flight (H2D), then leaf kernel + tree reduce + BFS image, D2H image --
      swept over gather threads and chunk size;
  (b) device-resident kernels with the transfers alone: pinned H2D of the values,
      the tree, D2H of the 44 MB image -- i.e. what a caller that already keeps
      values in pinned memory pays.
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from nakevaleng_amd import _lib  # noqa: E402
from oracle import oracle_c as oc  # noqa: E402


def main():
    L = _lib.lib()
    n, vlen = 1 << 20, 4096
    host = oc.splitmix64_bytes(n * vlen, 0x6E616B65)
    off = np.arange(n, dtype=np.uint64) * vlen
    lens = np.full(n, vlen, np.uint64)
    img = np.zeros(L.nkv_bfs_size(n), np.uint8)
    ctx = _lib.Context(0)
    ctx.set_option(_lib.NKV_OPT_BUCKET, 0)  # uniform values: fused path
    res = {}
    gib = n * vlen / 2**30
    cpu = next((ln.split(":", 1)[1].strip() for ln in open("/proc/cpuinfo") if ln.startswith("model name")), "?")
    print(f"host: {cpu}, os.cpu_count()={os.cpu_count()}, sched_getaffinity={len(os.sched_getaffinity(0))}")
    sweep = []
    for threads in (1, 4, 8, 16):
        for chunk_mib in (8, 32, 64):
            if threads == 1 and chunk_mib != 32:
                continue
            ctx.set_option(_lib.NKV_OPT_HOST_THREADS, threads)
            ctx.set_option(_lib.NKV_OPT_STAGE_CHUNK, chunk_mib << 20)
            ts = []
            for it in range(4):
                t0 = time.perf_counter()
                _lib.check(L.nkv_tree_from_values(ctx.h, _lib.p8(host), _lib.p64(off), _lib.p64(lens), n, None,
                                                  None, _lib.p8(img)))
                if it:
                    ts.append(time.perf_counter() - t0)
            sweep.append((min(ts), threads, chunk_mib))
            print(f"(a) host API nkv_tree_from_values, {threads:2d} gather threads, {chunk_mib:2d} MiB chunks: "
                  f"{min(ts)*1e3:.1f} ms  {gib/min(ts):.1f} GiB/s", flush=True)
    res["a_host_api"] = [min(sweep)[0]]
    best = min(sweep)
    ctx.set_option(_lib.NKV_OPT_HOST_THREADS, best[1])
    ctx.set_option(_lib.NKV_OPT_STAGE_CHUNK, best[2] << 20)
    # (b) pinned values -> device, device tree + image, image -> pinned
    s = torch.cuda.current_stream()
    ctx.set_stream(s.cuda_stream)
    pin = torch.from_numpy(host).pin_memory()
    d = torch.empty(n * vlen, dtype=torch.uint8, device="cuda")
    nodes = torch.empty(L.nkv_total_nodes(n) * 20, dtype=torch.uint8, device="cuda")
    dimg = torch.empty(img.size, dtype=torch.uint8, device="cuda")
    himg = torch.empty(img.size, dtype=torch.uint8).pin_memory()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
    for it in range(6):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ev[0].record(s)
        d.copy_(pin, non_blocking=True)
        ev[1].record(s)
        _lib.check(L.nkv_tree_from_strided_dev(ctx.h, d.data_ptr(), vlen, vlen, n, nodes.data_ptr()))
        _lib.check(L.nkv_bfs_image_dev(ctx.h, nodes.data_ptr(), n, dimg.data_ptr()))
        ev[2].record(s)
        himg.copy_(dimg, non_blocking=True)
        ev[3].record(s)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        if it:
            res.setdefault("b_pinned", []).append(dt)
            res.setdefault("b_h2d_ms", []).append(ev[0].elapsed_time(ev[1]))
            res.setdefault("b_compute_ms", []).append(ev[1].elapsed_time(ev[2]))
            res.setdefault("b_d2h_ms", []).append(ev[2].elapsed_time(ev[3]))
    assert himg.numpy().tobytes() == img.tobytes(), "host API and device path images differ"
    a = min(res["a_host_api"])
    b = min(res["b_pinned"])
    print(f"(a) best host API nkv_tree_from_values: {a*1e3:.1f} ms  {gib/a:.1f} GiB/s "
          f"({best[1]} threads, {best[2]} MiB chunks; gather + H2D + tree + image + D2H)")
    print(f"(b) pinned H2D + device tree/image + D2H image: {b*1e3:.1f} ms  {gib/b:.1f} GiB/s  "
          f"[H2D {min(res['b_h2d_ms']):.1f} ms = {n*vlen/min(res['b_h2d_ms'])/1e6:.1f} GB/s, "
          f"compute {min(res['b_compute_ms']):.2f} ms, D2H {min(res['b_d2h_ms']):.2f} ms]")
    ctx.close()


if __name__ == "__main__":
    main()
