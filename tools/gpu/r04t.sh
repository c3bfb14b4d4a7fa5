#!/bin/bash
# round 4 (t): URM forward megakernel LDS-layout variants (tile pitch, V transpose by MFMA)
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
for v in "" tools/alt/libg2048_urm_vtr.so tools/alt/libg2048_urm_tp196.so tools/alt/libg2048_urm_both.so tools/alt/libg2048_urm_tp204.so; do
  echo "== ${v:-in-tree}"
  G2048_LIB=$v timeout -k 10 120 python3 tools/time_urm.py 65536 64 10 2>&1 | tail -1
  rc=$?; [ $rc -ne 0 ] && exit $rc
done
