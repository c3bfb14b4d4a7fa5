# round 4: (1) GPU parity tests of the changed kernels (env kLine12 addressing, scalar LayerNorm
# epilogues, 8-wave fused passes, multi-CU Muon); (2) A/B timings of the fused passes (round-3 build,
# this tree, variants in tools/alt) and of the Muon step by CU count; (3) headline bench; (4) PMC.
# Ordinary test failures do not stop the script; a crash / abort / time limit does.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/r04b
export TMPDIR=/tmp
fatal() { case $1 in 124|134|137|139) echo "FATAL rc=$1 in $2"; exit $1;; esac; }
T="python -u -m pytest -m gpu -q --timeout 200 --timeout-method thread"
timeout -k 10 300 $T tests/test_gpu_env.py tests/test_gpu_policy_rollout.py > gpurun_out/r04b/tests_env.log 2>&1
rc=$?; echo "env/rollout tests rc=$rc"; tail -2 gpurun_out/r04b/tests_env.log; fatal $rc env
timeout -k 10 400 $T tests/test_gpu_ppo_fused.py -k "not muon" > gpurun_out/r04b/tests_fused.log 2>&1
rc=$?; echo "fused tests rc=$rc"; tail -2 gpurun_out/r04b/tests_fused.log; grep -E "^FAILED" gpurun_out/r04b/tests_fused.log | head; fatal $rc fused
timeout -k 10 300 $T tests/test_gpu_ppo_fused.py -k "muon" > gpurun_out/r04b/tests_muon.log 2>&1
rc=$?; echo "muon tests rc=$rc"; tail -2 gpurun_out/r04b/tests_muon.log; grep -E "^FAILED|Error" gpurun_out/r04b/tests_muon.log | head; fatal $rc muon
for v in r03 cur unrolled w4 fp8bp4; do
  lib=tools/alt/libg2048_$v.so; [ $v = cur ] && lib=2048-ppo_amd/g2048/libg2048.so
  echo "== $v" >> gpurun_out/r04b/time.log
  timeout -k 10 120 env G2048_LIB=$lib python -u tools/time_fused.py 4096,65536,262144 >> gpurun_out/r04b/time.log 2>&1
  rc=$?; fatal $rc "time $v"
done
grep -v amdgpu.ids gpurun_out/r04b/time.log
for parts in 1 8 12; do
  G2048_MUON_PARTS=$parts timeout -k 10 120 python -u tools/time_muon.py - 196 >> gpurun_out/r04b/time_muon.log 2>&1
  rc=$?; echo "parts=$parts rc=$rc" >> gpurun_out/r04b/time_muon.log; fatal $rc "muon $parts"
done
grep -v amdgpu.ids gpurun_out/r04b/time_muon.log
timeout -k 10 300 python3 bench.py --cpu-seconds 0 --urm-steps 0 --single-steps 0 --sweep '' > gpurun_out/r04b/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -c 2500 gpurun_out/r04b/bench.log; fatal $rc bench
TAG=r04b_fused bash tools/pmc_kernel.sh python3 tools/time_fused.py 65536 > gpurun_out/r04b/pmc.log 2>&1
echo "pmc rc=$?"; cat gpurun_out/r04b/pmc.log
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES -T --output-format csv -d gpurun_out/r04b/icache -o run -- python3 tools/time_fused.py 65536 > gpurun_out/r04b/icache.log 2>&1
echo "icache rc=$?"; python3 tools/pmc_table.py gpurun_out/r04b/icache mlp_ 2>&1 | head -40
