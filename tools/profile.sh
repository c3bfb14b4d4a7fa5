#!/bin/bash
# rocprofv3 passes for the bench command (GPU box): kernel trace + stats of the default line, then
# separate PMC passes of the rollout leg (FETCH_SIZE and WRITE_SIZE do not fit one pass on gfx950;
# two SQ passes of 8 counters).  No sys/hip tracing with PMC.  Summarise with
#   python tools/summarize_profile.py gpurun_out/prof_$TAG profiles/$TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
TAG=${TAG:-r02}
ARGS=${ARGS:---steps 20 --warmup 3 --cpu-seconds 0 --sweep=}
PMC_ARGS=${PMC_ARGS:---steps 4 --warmup 1 --cpu-seconds 0 --single-steps 64 --train-iters 0 --urm-steps 0 --sweep=}
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
pass() {  # pass <name> <rocprofv3 options...>
  local name=$1; shift
  timeout -k 10 300 rocprofv3 "$@" -T --output-format csv -d $OUT/$name -o run -- python3 bench.py $PMC_ARGS > $OUT/$name.log 2>&1
  local rc=$?; echo "$name rc=$rc"; return $rc
}
timeout -k 10 600 rocprofv3 --kernel-trace --stats -T --output-format csv -d $OUT/trace -o run -- python3 bench.py $ARGS > $OUT/trace.log 2>&1
rc=$?; echo "trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
find $OUT/trace -name "*kernel_trace.csv" -size +20M -delete  # keep gpurun_out under its copy-back cap
pass fetch --pmc FETCH_SIZE || exit $?
pass write --pmc WRITE_SIZE || exit $?
pass sqa --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES || exit $?
pass sqb --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE
