"""Per-kernel mean of every counter in a directory of rocprofv3 --pmc csv files."""
import csv
import glob
import os
import sys
from collections import defaultdict

d = sys.argv[1]
for f in sorted(glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)):
    acc = defaultdict(list)
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"]
        if "k_leaf" not in name:
            continue
        acc[(name.split("(")[0], r["Counter_Name"])].append(float(r["Counter_Value"]))
    for (k, c), v in sorted(acc.items()):
        print(f"{os.path.basename(f)[:28]:28s} {k[:24]:24s} {c:24s} {sum(v) / len(v):16.1f} (n={len(v)})")
