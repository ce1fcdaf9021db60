#!/usr/bin/env python3
"""profiles/pmc_traffic_<tag>.json from tools/pmc_config.sh's passes
(gpurun_out/pmc_<tag>/{req,fetch,write,sizes}_counter_collection.csv): the
per-dispatch TCC means of one config's leaf kernel and its HBM bytes per
launch, read the way profiles/pmc_traffic.json reads cfg2's (tools/pmc_traffic.py):
read bytes = 32 x RDREQ_32B + 64 x _64B + 128 x _128B (memory-side requests,
Infinity-Cache hits included, so an upper bound on HBM reads), plus WRITE_SIZE.

    python tools/pmc_traffic_cfg.py <tag> <kernel name prefix> <payload bytes> <leaves>
"""
import collections
import csv
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
tag, kernel, payload, leaves = sys.argv[1], sys.argv[2], int(sys.argv[3]), int(sys.argv[4])
src = os.path.join(ROOT, "gpurun_out", f"pmc_{tag}")
vals = collections.defaultdict(list)
for name in ("req", "fetch", "write", "sizes"):
    path = os.path.join(src, f"{name}_counter_collection.csv")
    with open(path) as f:
        for r in csv.DictReader(f):
            if r["Kernel_Name"].startswith(kernel):
                vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
mean = {k: sum(v) / len(v) for k, v in vals.items()}
read_bytes = 32 * mean["TCC_EA0_RDREQ_32B"] + 64 * mean["TCC_EA0_RDREQ_64B"] + 128 * mean["TCC_EA0_RDREQ_128B"]
out = {
    "about": f"rocprofv3 --pmc passes (tools/pmc_config.sh {tag}), kernel {kernel}: per-dispatch means over "
             f"{len(vals['TCC_EA0_RDREQ'])} dispatches",
    "config": tag,
    "leaves": leaves,
    "algorithmic_bytes_per_launch": payload,
    "kernel": kernel,
    "counters": {k: v for k, v in sorted(mean.items())},
    "read_bytes_per_launch": read_bytes,
    "hbm_read_bytes_bounds_per_launch": [mean["TCC_EA0_RDREQ"] * 64, mean["TCC_EA0_RDREQ"] * 128],
    "hbm_bytes_per_launch": read_bytes + 1024 * mean["WRITE_SIZE"],
    "traffic_over_payload": (read_bytes + 1024 * mean["WRITE_SIZE"]) / payload,
}
dst = os.path.join(ROOT, "profiles", f"pmc_traffic_{tag}.json")
with open(dst, "w") as f:
    json.dump(out, f, indent=1)
print(json.dumps(out, indent=1))
