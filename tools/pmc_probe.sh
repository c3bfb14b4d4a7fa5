#!/bin/bash
# SQ and memory counters of a probe executable (separate PMC passes, kernel-trace only):
#   pmc_probe.sh <tag> <cmd...>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
TAG=$1; shift
OUT=gpurun_out/pmc_$TAG
mkdir -p $OUT
timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD -T --output-format csv -d $OUT/a -o run -- "$@" > $OUT/a.log 2>&1
rc=$?; echo "pass a rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE -T --output-format csv -d $OUT/b -o run -- "$@" > $OUT/b.log 2>&1
rc=$?; echo "pass b rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE -T --output-format csv -d $OUT/c -o run -- "$@" > $OUT/c.log 2>&1
rc=$?; echo "pass c rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 rocprofv3 --pmc WRITE_SIZE -T --output-format csv -d $OUT/d -o run -- "$@" > $OUT/d.log 2>&1
rc=$?; echo "pass d rc=$rc"; exit $rc
