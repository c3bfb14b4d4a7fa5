"""Per-kernel mean durations of a tools/trace_muon.sh trace, split by time_muon.py's phases
(3 warmup steps, then 50 steps each at ns_steps = 5 / 0 / 1 / 5)."""
import collections
import csv
import statistics
import sys

rows = sorted(csv.DictReader(open(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/mtrace/run_kernel_trace.csv")),
              key=lambda r: int(r["Start_Timestamp"]))
rows = [r for r in rows if "rocclr" not in r["Kernel_Name"] and "elementwise" not in r["Kernel_Name"]
        and "reduce_kernel" not in r["Kernel_Name"] and "Cat" not in r["Kernel_Name"]]
steps = [i for i, r in enumerate(rows) if "grad_sumsq" in r["Kernel_Name"]]
phases = (("ns5", 3, 53), ("ns0", 53, 103), ("ns1", 103, 153))
for name, a, b in phases:
    d = collections.defaultdict(list)
    span = []
    for s in range(a, b):
        lo, hi = steps[s], steps[s + 1] if s + 1 < len(steps) else len(rows)
        for r in rows[lo:hi]:
            k = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0]
            d[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
        span.append((int(rows[hi - 1]["End_Timestamp"]) - int(rows[lo]["Start_Timestamp"])) / 1e3)
    print(name, "step span %.1f us:" % statistics.mean(span), ", ".join(f"{k} {statistics.mean(v):.1f}" for k, v in d.items()))
