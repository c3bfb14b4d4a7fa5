#!/bin/bash
# round 4 (s): SQ counters of the URM forward megakernel
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r04s; mkdir -p $O
export TMPDIR=/tmp
TAG=r04s_urmfwd bash tools/pmc_kernel.sh python3 tools/time_urm.py 65536 64 3 > $O/pmc.log 2>&1
echo "pmc rc=$?"; cat $O/pmc.log
python3 tools/pmc_table.py gpurun_out/pmck_r04s_urmfwd urm_forward 2>&1 | head -40
