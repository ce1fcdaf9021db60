#!/usr/bin/env python3
"""A/B of the resident service's request mailbox (NKV_OPT_SERVICE_MAILBOX 0:
device memory the host stores to through the large BAR; 1: host memory),
interleaved in ONE process so that box and placement noise falls on both forms
alike: each round switches the form (the service restarts, so each round is a
fresh launch and placement), warms up, then times `--calls` default-size
flushes (10 values of 1..200 B, no image, and 40 values with the image) through
nkv_tree_from_values; medians per round and over all rounds, roots checked
against the oracle.  A watchdog ends the process after --limit seconds.

    python tools/svc_ab.py [--rounds 8] [--calls 400] [--limit 150]
"""
import faulthandler
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def arg(name, default):
    return int(sys.argv[sys.argv.index(name) + 1]) if name in sys.argv else default


def main():
    limit = arg("--limit", 150)
    faulthandler.dump_traceback_later(limit, exit=True)
    import numpy as np
    from nakevaleng_amd import _lib
    from oracle import oracle_c as oc
    L = _lib.lib()
    ctx = _lib.Context(0)
    ctx.set_option(_lib.NKV_OPT_SMALL_PATH, 3)
    rng = np.random.default_rng(11)
    shapes = []
    for n, with_img in ((10, False), (40, True)):
        ln = rng.integers(1, 201, n).astype(np.uint64)
        off = np.zeros(n, np.uint64)
        off[1:] = np.cumsum(ln[:-1])
        base = np.frombuffer(rng.bytes(int(ln.sum()) + 1), np.uint8).copy()
        want = oc.tree_from_digests(oc.leaf_hashes(base, off, ln))[-1].tobytes()
        img = np.zeros(L.nkv_bfs_size(n), np.uint8)
        shapes.append((n, with_img, base, off, ln, want, img))
    rounds, calls = arg("--rounds", 8), arg("--calls", 400)
    res = {0: {s[0]: [] for s in shapes}, 1: {s[0]: [] for s in shapes}}
    for r in range(rounds):
        for mb in ((0, 1) if r % 2 == 0 else (1, 0)):
            ctx.set_option(_lib.NKV_OPT_SERVICE_MAILBOX, mb)
            for n, with_img, base, off, ln, want, img in shapes:
                root = np.zeros(20, np.uint8)
                ts = []
                for k in range(calls + 50):
                    t0 = time.perf_counter()
                    _lib.check(L.nkv_tree_from_values(ctx.h, _lib.p8(base), _lib.p64(off), _lib.p64(ln), n,
                                                      _lib.p8(root), None, _lib.p8(img) if with_img else None))
                    if k >= 50:
                        ts.append((time.perf_counter() - t0) * 1e6)
                assert root.tobytes() == want, (mb, n)
                med = float(np.median(ts))
                res[mb][n].append(med)
                # the same calls traced: the service's own phase times (stamps at 100 MHz)
                ctx.small_service_trace(True)
                st_ = []
                for _ in range(60):
                    _lib.check(L.nkv_tree_from_values(ctx.h, _lib.p8(base), _lib.p64(off), _lib.p64(ln), n,
                                                      _lib.p8(root), None, _lib.p8(img) if with_img else None))
                    st_.append(ctx.small_service_trace(True))
                ctx.small_service_trace(False)
                rt = np.array(st_[10:], np.float64)[:, 0::2]
                ph = {k: round(float(np.median(rt[:, j1] - rt[:, j0])) / 100.0, 2)
                      for k, j0, j1 in (("stage_in", 0, 1), ("leaves", 1, 2), ("levels", 2, 3), ("signal", 3, 4))}
                st = ctx.small_service_state()
                print(f"round {r} mailbox {mb} (dev {st['mailbox_dev']}) n={n}: median {med:.2f} us, "
                      f"p10 {np.percentile(ts, 10):.2f}, p90 {np.percentile(ts, 90):.2f}; phases {ph}; "
                      f"xcc {st['xcc']} se {st['se']} sh {st['sh']} cu {st['cu']} simd {st['simd']}", flush=True)
    out = {"rounds": rounds, "calls": calls}
    for mb in (0, 1):
        for n in res[mb]:
            v = res[mb][n]
            out[f"mailbox{mb}_n{n}"] = {"median_of_round_medians_us": round(float(np.median(v)), 2),
                                        "min": round(min(v), 2), "max": round(max(v), 2)}
    print("ab " + json.dumps(out), flush=True)
    ctx.close()
    faulthandler.cancel_dump_traceback_later()


if __name__ == "__main__":
    main()
