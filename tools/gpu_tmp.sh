set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pt.log 2>&1; rc=$?; tail -3 gpurun_out/pt.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u tools/ab_propose.py --config cfg2 > gpurun_out/abp.log 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/abp.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u tools/ab_propose.py --config cfg5 > gpurun_out/abp5.log 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/abp5.log; exit $rc
