cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; O=gpurun_out/r06c; mkdir -p $O
timeout -k 10 240 rocprofv3 --kernel-trace -T --output-format csv -d $O/trace -o run -- python3 bench.py --steps 3 --warmup 1 --cpu-seconds 0 --urm-steps 0 --single-steps 0 --sweep= --train-iters 1 --train-warmup 1 > $O/trace.log 2>&1
echo rc=$?
f=$(find $O/trace -name "*kernel_trace.csv" | head -1)
python3 tools/timeline.py $f mlp_back_kernel > $O/timeline.txt; cat $O/timeline.txt
python3 - $f <<'PY'
import csv,sys
rows=sorted(csv.DictReader(open(sys.argv[1])),key=lambda r:int(r["Start_Timestamp"]))
p=[r for r in rows if r["Kernel_Name"].startswith("mlp_pass") or "mlp_pass_kernel" in r["Kernel_Name"]]
names={}
for r in p:
    k=r["Kernel_Name"][:60]; d=(int(r["End_Timestamp"])-int(r["Start_Timestamp"]))/1000
    names.setdefault(k,[]).append(d)
for k,v in names.items(): print(k, len(v), sum(v)/len(v))
PY
find $O/trace -name "*kernel_trace.csv" -size +20M -delete
