set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "propose or nms" -x -q --timeout 120 --timeout-method thread > gpurun_out/pt.log 2>&1; rc=$?; tail -2 gpurun_out/pt.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u tools/prop_timeline.py cfg2 > gpurun_out/ptl.log 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/ptl.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u tools/ab_propose.py --config cfg2 --paths fused,lazy > gpurun_out/abp.log 2>&1; rc=$?; grep -A3 '"fused"' gpurun_out/abp.log; exit $rc
