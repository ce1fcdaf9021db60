#!/usr/bin/env python3
"""Counters of the resident service (run under rocprofv3 --pmc): --calls
default-size flushes (10 values of 1..200 B, no image) through
NKV_OPT_SMALL_PATH 3, then the service is left to exit on its idle timeout.
With counter collection each service launch serves few requests (the
profiler wraps every dispatch), so the per-dispatch counters read per request.
A watchdog ends the process after --limit seconds.

    rocprofv3 --pmc SQC_ICACHE_MISSES SQC_ICACHE_HITS -d DIR -- python3 tools/svc_pmc.py
"""
import faulthandler
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    limit = int(sys.argv[sys.argv.index("--limit") + 1]) if "--limit" in sys.argv else 50
    calls = int(sys.argv[sys.argv.index("--calls") + 1]) if "--calls" in sys.argv else 40
    faulthandler.dump_traceback_later(limit, exit=True)
    import numpy as np
    from nakevaleng_amd import _lib
    from oracle import oracle_c as oc
    L = _lib.lib()
    ctx = _lib.Context(0)
    ctx.set_option(_lib.NKV_OPT_SMALL_PATH, 3)
    rng = np.random.default_rng(11)
    n = 10
    ln = rng.integers(1, 201, n).astype(np.uint64)
    off = np.zeros(n, np.uint64)
    off[1:] = np.cumsum(ln[:-1])
    base = np.frombuffer(rng.bytes(int(ln.sum()) + 1), np.uint8).copy()
    want = oc.tree_from_digests(oc.leaf_hashes(base, off, ln))[-1].tobytes()
    root = np.zeros(20, np.uint8)
    t0 = time.perf_counter()
    for _ in range(calls):
        _lib.check(L.nkv_tree_from_values(ctx.h, _lib.p8(base), _lib.p64(off), _lib.p64(ln), n, _lib.p8(root),
                                          None, None))
    assert root.tobytes() == want
    st = ctx.small_service_state()
    print(f"{calls} calls in {time.perf_counter() - t0:.3f} s; state {st}", flush=True)
    time.sleep(0.1)  # the service leaves on its idle timeout
    ctx.close()
    faulthandler.cancel_dump_traceback_later()


if __name__ == "__main__":
    main()
