#!/usr/bin/env python3
"""Copy the rocprofv3 summaries of tools/profile_r01.sh from gpurun_out/prof into
profiles/ (kernel stats CSV + the JSON line the profiled command printed)."""
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "gpurun_out", "prof")
DST = os.path.join(ROOT, "profiles")
tag = sys.argv[1] if len(sys.argv) > 1 else "r01"
for name in ("cfg2", "cfg3", "records", "records_verify", "crc", "bloom"):
    stats = os.path.join(SRC, f"{name}_kernel_stats.csv")
    line = os.path.join(SRC, f"{name}.json")
    if os.path.exists(stats):
        shutil.copy(stats, os.path.join(DST, f"{tag}_{name}_kernel_stats.csv"))
    if os.path.exists(line):
        shutil.copy(line, os.path.join(DST, f"{tag}_{name}_bench_under_rocprof.json"))
    print(name, "ok" if os.path.exists(stats) else "missing")
