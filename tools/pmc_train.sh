#!/bin/bash
# rocprofv3 passes over the bench's training legs (GPU box): the MLP train iteration (fused policy
# rollout + RTG + D4 up-sampling + the kernel-written PPO update, h 196, 65 536 envs x T 64) and,
# with URM=1, the GameURM leg.  One kernel-trace pass, then FETCH / WRITE / two SQ passes (gfx950:
# FETCH_SIZE and WRITE_SIZE do not share a pass; at most 8 SQ counters per pass).  Summarise with
#   python tools/summarize_profile.py gpurun_out/ptrain_$TAG profiles/$TAG/train
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
TAG=${TAG:-r03}
URMS=${URM:+8}
ARGS=${ARGS:---steps 2 --warmup 1 --cpu-seconds 0 --single-steps 0 --train-iters 1 --train-warmup 1 --urm-steps ${URMS:-0} --sweep=}
OUT=gpurun_out/ptrain_$TAG
mkdir -p $OUT
# progress line every 50 s (PMC passes write nothing until they finish): the pass output sizes so far
( while true; do sleep 50; echo "$(date +%T) $(du -sk $OUT 2>/dev/null | cut -f1) KiB in $OUT"; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
pass() {  # pass <name> <rocprofv3 options...>
  local name=$1; shift
  timeout -k 10 300 rocprofv3 "$@" -T --output-format csv -d $OUT/$name -o run -- python3 bench.py $ARGS > $OUT/$name.log 2>&1
  local rc=$?; echo "$name rc=$rc"; return $rc
}
pass trace --kernel-trace --stats || exit $?
find $OUT/trace -name "*kernel_trace.csv" -size +20M -delete
pass fetch --pmc FETCH_SIZE || exit $?
pass write --pmc WRITE_SIZE || exit $?
pass sqa --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES || exit $?
pass sqb --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU GRBM_GUI_ACTIVE || exit $?
pass sqc --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_MISC
