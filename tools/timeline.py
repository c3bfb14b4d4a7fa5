"""One minibatch's kernel timeline from a rocprofv3 --kernel-trace CSV (the span between the last
two launches of the marker kernel): python tools/timeline.py <kernel_trace.csv> [marker]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
marker = sys.argv[2] if len(sys.argv) > 2 else "obs_gather"
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if marker in r["Kernel_Name"]]
i0, i1 = idx[-2], idx[-1]
t0 = int(rows[i0]["Start_Timestamp"])
prev_end, tot = t0, 0
for r in rows[i0:i1]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    n = r["Kernel_Name"].replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0][:70]
    print(f"{(s - t0) / 1000:8.1f} gap={(s - prev_end) / 1000:5.1f} dur={(e - s) / 1000:6.1f}  {n}")
    tot += e - s
    prev_end = e
print("span", (int(rows[i1]["Start_Timestamp"]) - t0) / 1000, "us; kernel sum", tot / 1000, "us")
