set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "roi_pool" -x -q --timeout 120 --timeout-method thread > gpurun_out/pt.log 2>&1; rc=$?; tail -3 gpurun_out/pt.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u tools/ab_roi_pool.py --config cfg2 --rounds ${ROUNDS:-5} --variants ${AB} > gpurun_out/ab.log 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/ab.log | grep -v 'GBps\|us_min'; exit $rc
