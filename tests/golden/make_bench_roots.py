#!/usr/bin/env python3
"""Generate tests/golden/bench_roots.json (committed) -- run in the build container.

The expected roots of bench.py's synthetic tables, so that every rank of a
`bench.py --gpus N` run checks its own root against a fixed value without
running the oracle on the GPU box:

  sstable4k[r][t]  root of table t on rank r: 1 Mi values x 4 KiB, value i at
                   byte 4096 i of splitmix64 bytes with seed 0x6e616b65 + r +
                   7919 t (bench.py build_tables), r = 0..7, t = 0..3 (t > 0:
                   the extra tables of --tables / --config runs4);
  one_tree[N]      root of ONE tree over the leaves of ranks 0..N-1 (t = 0)
                   in rank order (bench.py --config one_tree, the split over N
                   GPUs), N = 1..8;
  small[r]         the same shape rule at 1 Ki values x 1 KiB (BASELINE
                   configs[0]'s size) for the CPU tests of the verification;
  records[r]       bench.py --config records / records_verify: 1 Mi serialized
                   4096-byte records (16-byte key) over splitmix64 bytes with
                   seed 0x6e616b65 + r, leaves = the Values at +46 (the header
                   fields the bench writes lie outside them);
  mixed[r]         bench.py --config mixed: BASELINE configs[2]'s 4 GiB of
                   log-uniform 64 B - 64 KiB values (bench.mixed_lengths, numpy's
                   default_rng, seed 0x6e616b66 + r) over splitmix64 bytes of the
                   same seed;
  config4[r]       BASELINE configs[4]'s per-GPU table: 8 Mi values x 4 KiB (32
                   GiB) with seed 0x6e616b65 + r, generated and hashed 1 Mi values
                   at a time (the oracle's stream at a byte offset).

Every root comes from oracle/merkle_oracle.c (the C restatement of
ds/merkletree: leaf = SHA-1(value), merkletree.go:31-64's build), which the
CPU suite pins against the FIPS SHA-1 vectors and the literal Python
restatement (tests/test_oracle.py).  Tree level: parity unpinned, as for every
fixture in this directory.

    python tests/golden/make_bench_roots.py [--threads 8] [--only config4]
    (--only SECTION recomputes one section into the existing file)
"""
import argparse
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from oracle import oracle_c as oc  # noqa: E402

SEED = 0x6E616B65
TABLE_SEED_STEP = 7919
RANKS, TABLES = 8, 4
OUT = os.path.join(HERE, "bench_roots.json")


def digests(n, vlen, seed, threads):
    data = oc.splitmix64_bytes(n * vlen, seed)
    d = oc.leaf_hashes_strided(data, vlen, vlen, n, threads=threads)
    del data
    return d


def config4(threads):
    import numpy as np
    n, vlen, chunk = 8 << 20, 4096, 1 << 20
    sec = {"leaves": n, "value_bytes": vlen, "roots": {}}
    t0 = time.time()
    for r in range(RANKS):
        d = np.empty((n, 20), np.uint8)
        for c in range(0, n, chunk):
            data = oc.splitmix64_bytes(chunk * vlen, SEED + r, first=c * vlen)
            d[c:c + chunk] = oc.leaf_hashes_strided(data, vlen, vlen, chunk, threads=threads)
            del data
        sec["roots"][str(r)] = oc.tree_from_digests(d)[-1].tobytes().hex()
        print(f"config4 rank {r}: {sec['roots'][str(r)]} ({time.time() - t0:.0f} s)", file=sys.stderr)
    return sec


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", type=int, default=os.cpu_count() or 8)
    ap.add_argument("--only", choices=["config4"], default=None)
    args = ap.parse_args()
    oc.build()
    if args.only:
        with open(OUT) as f:
            out = json.load(f)
        out["config4"] = config4(args.threads)
        with open(OUT, "w") as f:
            json.dump(out, f, indent=1)
            f.write("\n")
        return
    n, vlen = 1 << 20, 4096
    out = {
        "generator": "tests/golden/make_bench_roots.py (oracle/merkle_oracle.c)",
        "seed": SEED, "table_seed_step": TABLE_SEED_STEP,
        "sstable4k": {"leaves": n, "value_bytes": vlen, "roots": {}},
        "one_tree": {"leaves_per_rank": n, "value_bytes": vlen, "roots": {}},
        "small": {"leaves": 1024, "value_bytes": 1024, "roots": {}},
    }
    t0 = time.time()
    first = []  # rank r's table-0 leaf digests (the one-tree leaves)
    for r in range(RANKS):
        roots = []
        for t in range(TABLES):
            d = digests(n, vlen, SEED + r + TABLE_SEED_STEP * t, args.threads)
            roots.append(oc.tree_from_digests(d)[-1].tobytes().hex())
            if t == 0:
                first.append(d)
        out["sstable4k"]["roots"][str(r)] = roots
        print(f"rank {r}: {roots[0]} ({time.time() - t0:.0f} s)", file=sys.stderr)
    import numpy as np
    for N in range(1, RANKS + 1):
        out["one_tree"]["roots"][str(N)] = oc.tree_from_digests(np.concatenate(first[:N]))[-1].tobytes().hex()
    for r in range(RANKS):
        d = digests(1024, 1024, SEED + r, 1)
        out["small"]["roots"][str(r)] = oc.tree_from_digests(d)[-1].tobytes().hex()
    rb, ks = 4096, 16
    out["records"] = {"leaves": n, "record_bytes": rb, "key_bytes": ks, "roots": {}}
    for r in range(RANKS):
        stream = oc.splitmix64_bytes(n * rb, SEED + r)
        voff = np.arange(n, dtype=np.uint64) * rb + 30 + ks
        d = oc.leaf_hashes(stream, voff, np.full(n, rb - 30 - ks, np.uint64), threads=args.threads)
        del stream
        out["records"]["roots"][str(r)] = oc.tree_from_digests(d)[-1].tobytes().hex()
        print(f"records rank {r} ({time.time() - t0:.0f} s)", file=sys.stderr)
    import bench
    out["mixed"] = {"payload_bytes": 4 << 30, "seed": bench.SEED_MIXED, "roots": {}, "leaves": {}}
    for r in range(RANKS):
        lens, off = bench.mixed_lengths(4 << 30, bench.SEED_MIXED + r)
        data = oc.splitmix64_bytes(int(lens.sum()), bench.SEED_MIXED + r)
        d = oc.leaf_hashes(data, off, lens, threads=args.threads)
        del data
        out["mixed"]["roots"][str(r)] = oc.tree_from_digests(d)[-1].tobytes().hex()
        out["mixed"]["leaves"][str(r)] = int(len(lens))
        print(f"mixed rank {r} ({time.time() - t0:.0f} s)", file=sys.stderr)
    out["config4"] = config4(args.threads)
    with open(OUT, "w") as f:
        json.dump(out, f, indent=1)
        f.write("\n")
    print(f"wrote {OUT} in {time.time() - t0:.0f} s", file=sys.stderr)


if __name__ == "__main__":
    main()
