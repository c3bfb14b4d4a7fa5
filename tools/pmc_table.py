"""Print per-kernel averages of every counter in a tools/pmc_kernel.sh / pmc_sq.sh output directory.
    python tools/pmc_table.py gpurun_out/pmck_<tag> [kernel-substring]"""
import collections
import csv
import sys
from pathlib import Path

root, filt = Path(sys.argv[1]), (sys.argv[2] if len(sys.argv) > 2 else "")
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in root.rglob("*counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        if filt in r["Kernel_Name"]:
            acc[r["Kernel_Name"][:60]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, cs in sorted(acc.items()):
    print(k)
    for c, v in sorted(cs.items()):
        print(f"    {c:28s} {sum(v) / len(v):16.1f}  (n={len(v)})")
