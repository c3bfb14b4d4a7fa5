#!/bin/bash
# SQ counter passes (kernel-trace only, one PMC set per run) of an arbitrary python command:
#   TAG=x bash tools/pmc_kernel.sh python3 tools/time_rollout.py --reps 2
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
TAG=${TAG:-k}
OUT=gpurun_out/pmck_$TAG
mkdir -p $OUT
timeout -k 10 240 rocprofv3 --kernel-trace --stats -T --output-format csv -d $OUT/trace -o run -- "$@" > $OUT/trace.log 2>&1
rc=$?; echo "trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD -T --output-format csv -d $OUT/sqa -o run -- "$@" > $OUT/sqa.log 2>&1
rc=$?; echo "sqa rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 240 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_WR -T --output-format csv -d $OUT/sqb -o run -- "$@" > $OUT/sqb.log 2>&1
rc=$?; echo "sqb rc=$rc"; exit $rc
