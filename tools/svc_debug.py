#!/usr/bin/env python3
"""Diagnostic probe of the resident small-tree service (NKV_OPT_SMALL_PATH 3):
each call's wall time, result against the oracle and the mailbox state
(nkv_ctx_small_service_state), printed as it goes; a watchdog ends the process
after --limit seconds so a stuck call cannot hang the GPU job.

    python tools/svc_debug.py [--limit 60] [--modes 1,3] [--trace] [--mailbox 0|1]
"""
import faulthandler
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    limit = int(sys.argv[sys.argv.index("--limit") + 1]) if "--limit" in sys.argv else 60
    faulthandler.dump_traceback_later(limit, exit=True)
    import numpy as np
    from nakevaleng_amd import _lib
    from oracle import oracle_c as oc
    L = _lib.lib()
    ctx = _lib.Context(0)
    ctx.set_option(_lib.NKV_OPT_SMALL_PATH, 3)
    # --mailbox 1: the service's requests in host memory (NKV_OPT_SERVICE_MAILBOX)
    mailbox = int(sys.argv[sys.argv.index("--mailbox") + 1]) if "--mailbox" in sys.argv else 0
    ctx.set_option(_lib.NKV_OPT_SERVICE_MAILBOX, mailbox)
    print("mailbox option", mailbox, flush=True)
    rng = np.random.default_rng(3)
    print("state0", ctx.small_service_state(), flush=True)
    sizes = ([int(x) for x in sys.argv[sys.argv.index("--sizes") + 1].split(",")] if "--sizes" in sys.argv
             else [1, 2, 3, 10, 100, 1000, 10, 10])
    for n in sizes:
        ln = rng.integers(0, 200, n).astype(np.uint64)
        off = np.zeros(n, np.uint64)
        off[1:] = np.cumsum(ln[:-1])
        base = np.frombuffer(rng.bytes(int(ln.sum()) + 1), np.uint8).copy()
        root = np.zeros(20, np.uint8)
        nodes = np.zeros((L.nkv_total_nodes(n), 20), np.uint8)
        t0 = time.perf_counter()
        rc = L.nkv_tree_from_values(ctx.h, _lib.p8(base), _lib.p64(off), _lib.p64(ln), n, _lib.p8(root),
                                    _lib.p8(nodes), None)
        dt = (time.perf_counter() - t0) * 1e6
        want = oc.tree_from_digests(oc.leaf_hashes(base, off, ln))
        ok = rc == 0 and np.array_equal(nodes, want)
        print(f"n={n} rc={rc} ok={ok} us={dt:.1f} path={ctx.last_path()} state={ctx.small_service_state()}",
              flush=True)
        if not ok and rc == 0:
            bad = np.nonzero((nodes != want).any(axis=1))[0]
            print(f"  wrong nodes: {len(bad)} of {len(want)}, first {bad[:8].tolist()}", flush=True)
    # steady-state latency of the default flush (10 values <= 200 B) and
    # compaction (40) shapes, per small-path mode (--modes, default 3)
    modes = [int(m) for m in (sys.argv[sys.argv.index("--modes") + 1] if "--modes" in sys.argv else "3").split(",")]
    for mode in modes:
        ctx.set_option(_lib.NKV_OPT_SMALL_PATH, mode)
        for n in (10, 40):
            ln = rng.integers(1, 201, n).astype(np.uint64)
            off = np.zeros(n, np.uint64)
            off[1:] = np.cumsum(ln[:-1])
            base = np.frombuffer(rng.bytes(int(ln.sum()) + 1), np.uint8).copy()
            root = np.zeros(20, np.uint8)
            want = oc.tree_from_digests(oc.leaf_hashes(base, off, ln))[-1].tobytes()
            ts = []
            for _ in range(300):
                t0 = time.perf_counter()
                _lib.check(L.nkv_tree_from_values(ctx.h, _lib.p8(base), _lib.p64(off), _lib.p64(ln), n,
                                                  _lib.p8(root), None, None))
                ts.append((time.perf_counter() - t0) * 1e6)
            assert root.tobytes() == want, (mode, n)
            ts.sort()
            print(f"mode {mode} n={n} x300: median {ts[150]:.1f} us, p10 {ts[30]:.1f}, p90 {ts[270]:.1f}; "
                  f"state={ctx.small_service_state()}", flush=True)
    # where a request's time goes inside the service (--trace): the stamps of
    # every request, phase medians in us and the shader clock over each phase
    if "--trace" in sys.argv:
        import json
        ctx.set_option(_lib.NKV_OPT_SMALL_PATH, 3)
        for n, lo, hi, with_img in ((10, 1, 200, False), (10, 1, 200, True), (40, 1, 200, True),
                                    (256, 1, 200, True)):
            img = np.zeros(L.nkv_bfs_size(n), np.uint8)
            ln = rng.integers(lo, hi + 1, n).astype(np.uint64)
            off = np.zeros(n, np.uint64)
            off[1:] = np.cumsum(ln[:-1])
            base = np.frombuffer(rng.bytes(int(ln.sum()) + 1), np.uint8).copy()
            root = np.zeros(20, np.uint8)
            ctx.small_service_trace(True)
            st, walls = [], []
            for _ in range(200):
                t0 = time.perf_counter()
                _lib.check(L.nkv_tree_from_values(ctx.h, _lib.p8(base), _lib.p64(off), _lib.p64(ln), n,
                                                  _lib.p8(root), None, _lib.p8(img) if with_img else None))
                walls.append((time.perf_counter() - t0) * 1e6)
                st.append(ctx.small_service_trace(True))
            ctx.small_service_trace(False)
            a = np.array(st[20:], np.float64)
            rt, mt = a[:, 0::2], a[:, 1::2]
            out = {"n": n, "value_bytes": [lo, hi], "image": with_img,
                   "wall_us_median": round(float(np.median(walls[20:])), 2)}
            phases = [("request_and_stage_in", 0, 1), ("leaves", 1, 2), ("levels_and_image", 2, 3),
                      ("signal", 3, 4), ("seen_to_signal", 0, 4), ("levels", 2, 5)]
            if rt[:, 6].min() > 0:  # an image was built
                phases += [("image_build", 5, 6), ("copy_out", 6, 3)]
            for name, j0, j1 in phases:
                us = (rt[:, j1] - rt[:, j0]) / 100.0
                ghz = (mt[:, j1] - mt[:, j0]) / np.maximum(rt[:, j1] - rt[:, j0], 1) * 100e6 / 1e9
                out[name] = {"us_median": round(float(np.median(us)), 2), "ghz_median": round(float(np.median(ghz)), 3)}
            print("trace " + json.dumps(out), flush=True)
    t0 = time.perf_counter()
    ctx.close()
    print(f"close {(time.perf_counter() - t0) * 1e3:.1f} ms", flush=True)
    faulthandler.cancel_dump_traceback_later()


if __name__ == "__main__":
    main()
