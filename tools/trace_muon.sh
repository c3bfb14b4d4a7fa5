#!/bin/bash
# kernel trace of tools/time_muon.py (GPU box): per-kernel durations by ns_steps setting
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/mtrace
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/mtrace -o run -- python3 tools/time_muon.py - ${H:-196} > gpurun_out/mtrace/log 2>&1
echo "trace rc=$?"
