#!/bin/bash
# rocprofv3 passes over tools/urm_pmc_step.py (GameURM training fwd+bwd + one-launch forward at
# 65 536 boards): kernel trace, FETCH / WRITE, two SQ passes.  Summarise with
#   python tools/summarize_profile.py gpurun_out/purm_$TAG profiles/$TAG/urm
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
TAG=${TAG:-r03}
OUT=gpurun_out/purm_$TAG
mkdir -p $OUT
( while true; do sleep 50; echo "$(date +%T) $(du -sk $OUT 2>/dev/null | cut -f1) KiB in $OUT"; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
pass() {  # pass <name> <rocprofv3 options...>
  local name=$1; shift
  timeout -k 10 240 rocprofv3 "$@" -T --output-format csv -d $OUT/$name -o run -- python3 tools/urm_pmc_step.py > $OUT/$name.log 2>&1
  local rc=$?; echo "$name rc=$rc"; return $rc
}
pass trace --kernel-trace --stats || exit $?
pass fetch --pmc FETCH_SIZE || exit $?
pass write --pmc WRITE_SIZE || exit $?
pass sqa --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES || exit $?
pass sqb --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU GRBM_GUI_ACTIVE || exit $?
pass sqc --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_MISC
