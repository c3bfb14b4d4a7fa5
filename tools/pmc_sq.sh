#!/bin/bash
# SQ instruction / stall counters for the env rollout kernel (one PMC pass each, kernel-trace only).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
TAG=${TAG:-sq}
OUT=gpurun_out/pmc_$TAG
mkdir -p $OUT
ARGS=${ARGS:---steps 3 --warmup 1 --cpu-seconds 0 --train-iters 0 --single-steps 0}
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES -T --output-format csv -d $OUT/a -o run -- python3 bench.py $ARGS > $OUT/a.log 2>&1
rc=$?; echo "pass a rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE -T --output-format csv -d $OUT/b -o run -- python3 bench.py $ARGS > $OUT/b.log 2>&1
rc=$?; echo "pass b rc=$rc"; exit $rc
