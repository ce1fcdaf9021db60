#!/usr/bin/env python3
"""Kernel statistics from a rocprofv3 SQLite database (`*_results.db`, the
default output of rocprofv3 --kernel-trace on this image) as the CSV
`--stats` writes: one row per kernel name with calls, total / average /
min / max duration in ns.  Optionally split one kernel's dispatches into
consecutive runs (``--split NAME:K``: K equal slices in launch order, e.g.
the shapes of tools/small_flush.cpp, each summarised apart, median too).

    python tools/rocpd_stats.py DB [--split NAME:K[:SKIP]] > stats.csv
"""
import argparse
import sqlite3
import statistics
import sys


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--split", default=None, help="NAME:K[:SKIP] -- K consecutive slices of NAME's dispatches, "
                                                  "the first SKIP of each dropped (warm-up)")
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    rows = c.execute("select name, duration from kernels order by start").fetchall()
    by = {}
    for name, d in rows:
        by.setdefault(name.split("(")[0], []).append(int(d))
    w = sys.stdout.write
    w("Name,Calls,TotalDurationNs,AverageNs,MinNs,MaxNs,MedianNs\n")
    for name, ds in sorted(by.items(), key=lambda kv: -sum(kv[1])):
        w(f"\"{name}\",{len(ds)},{sum(ds)},{sum(ds) / len(ds):.1f},{min(ds)},{max(ds)},{statistics.median(ds):.1f}\n")
    if a.split:
        parts = a.split.rsplit(":", 2)  # the kernel name itself holds "::"
        if len(parts) == 3 and parts[1].isdigit() and parts[2].isdigit():
            name, k, skip = parts[0], int(parts[1]), int(parts[2])
        else:
            name, k = a.split.rsplit(":", 1)
            k, skip = int(k), 0
        ds = by.get(name, [])
        per = len(ds) // k if k else 0
        w("Slice,Calls,AverageNs,MedianNs,P10Ns,P90Ns\n")
        for i in range(k):
            s = sorted(ds[i * per:(i + 1) * per][skip:])
            if not s:
                continue
            w(f"{i},{len(s)},{sum(s) / len(s):.1f},{statistics.median(s):.1f},{s[len(s) // 10]},"
              f"{s[9 * len(s) // 10]}\n")


if __name__ == "__main__":
    main()
