#!/bin/bash
# kernel trace of one GameURM fwd + bwd (tools/urm_pmc_step.py): every urm_linear_kernel dispatch
# with its template instance, grid and duration (which projection shapes are slowest)
cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp
O=gpurun_out/${TAG:-r06i}; mkdir -p $O
timeout -k 10 240 rocprofv3 --kernel-trace -T --output-format csv -d $O/utrace -o run -- python3 tools/urm_pmc_step.py > $O/utrace.log 2>&1
echo rc=$?
f=$(find $O/utrace -name "*kernel_trace.csv" | head -1)
python3 - $f <<'PY' | tee $O/urm_linear_shapes.txt
import csv, sys, collections
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
agg = collections.defaultdict(list)
for r in rows:
    k = r["Kernel_Name"]
    if not k.startswith("urm_") and "urm_" not in k:
        continue
    name = k.split("(")[0][:110]
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000
    agg[(name, r["Grid_Size"], r["LDS_Block_Size"], r.get("VGPR_Count"), r.get("Accum_VGPR_Count"))].append(d)
tot = sum(sum(v) for v in agg.values())
for key, v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
    print(f"{sum(v):9.1f} us {len(v):4d} x {sum(v)/len(v):7.1f}  grid {key[1]:>8} lds {key[2]:>6} vgpr {key[3]}/{key[4]}  {key[0]}")
print("total", tot)
PY
find $O/utrace -name "*kernel_trace.csv" -size +20M -delete
