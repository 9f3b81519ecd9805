# GPU call: full -m gpu suite, RoIPool forward A/B (cfg2), bench.  Each step
# has its own time limit; the script stops at the first abnormal exit.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 200 python -u tools/ab_roi_pool.py --config cfg2 --variants ${AB_VARIANTS:-sorted,px8sorted,px8s} > gpurun_out/ab.log 2>&1
rc=$?; echo "ab rc=$rc"; cat gpurun_out/ab.log | tail -30
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --steps 50 --warmup 10 --cpu-seconds 10 > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -3 gpurun_out/bench.log
