#!/bin/bash
# rocprofv3 passes over tools/time_muon.py (GPU box): kernel trace + SQ counter passes of the fused
# Muon + AdamW optimizer step at h 196.   bash tools/pmc_muon.sh; then
#   python tools/summarize_profile.py gpurun_out/pmuon_$TAG profiles/$TAG/muon
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
TAG=${TAG:-r03}
OUT=gpurun_out/pmuon_$TAG
mkdir -p $OUT
pass() {  # pass <name> <rocprofv3 options...>
  local name=$1; shift
  timeout -k 10 120 rocprofv3 "$@" -T --output-format csv -d $OUT/$name -o run -- python3 tools/time_muon.py - 196 quick > $OUT/$name.log 2>&1
  local rc=$?; echo "$name rc=$rc"; return $rc
}
pass trace --kernel-trace --stats || exit $?
pass sqa --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES || exit $?
pass sqb --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE || exit $?
pass sqc --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_MISC SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_SCA
