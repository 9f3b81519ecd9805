# GPU call: RoIPool forward A/B only (variants in $AB, config in $CFG).
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 200 python -u tools/ab_roi_pool.py --config ${CFG:-cfg2} --variants ${AB} > gpurun_out/ab.log 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/ab.log | grep -v '"GBps"\|us_min'; exit $rc
