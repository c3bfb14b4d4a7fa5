"""Per-kernel averages of the counters a tools/pmc_probe.sh run collected:
    python tools/pmc_table.py gpurun_out/pmc_<tag>"""
import collections
import csv
import sys
from pathlib import Path

root = Path(sys.argv[1])
vals = collections.defaultdict(lambda: collections.defaultdict(list))
for f in root.rglob("*counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0][-60:]
        vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, cs in sorted(vals.items()):
    print(k)
    for c, v in sorted(cs.items()):
        print(f"    {c:24s} {sum(v) / len(v):16.1f}  (n={len(v)})")
