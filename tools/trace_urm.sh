# kernel trace of tools/urm_pmc_step.py (GameURM training fwd+bwd x2 + one-launch forward x2)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/turm_${TAG:-r03}
mkdir -p $OUT
timeout -k 10 240 rocprofv3 --kernel-trace --stats -T --output-format csv -d $OUT -o run -- python3 tools/urm_pmc_step.py > $OUT/trace.log 2>&1
echo "trace rc=$?"
