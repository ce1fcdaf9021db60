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
                   configs[0]'s size) for the CPU tests of the verification.

Every root comes from oracle/merkle_oracle.c (the C restatement of
ds/merkletree: leaf = SHA-1(value), merkletree.go:31-64's build), which the
CPU suite pins against the FIPS SHA-1 vectors and the literal Python
restatement (tests/test_oracle.py).  Tree level: parity unpinned, as for every
fixture in this directory.

    python tests/golden/make_bench_roots.py [--threads 8]
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", type=int, default=os.cpu_count() or 8)
    args = ap.parse_args()
    oc.build()
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
    with open(OUT, "w") as f:
        json.dump(out, f, indent=1)
        f.write("\n")
    print(f"wrote {OUT} in {time.time() - t0:.0f} s", file=sys.stderr)


if __name__ == "__main__":
    main()
