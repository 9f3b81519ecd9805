# GPU-box script: parity tests, smoke, bench, rocprofv3 kernel stats of the SAME
# bench command, and PMC passes over the dominant kernel.  Writes gpurun_out/$TAG.
set -u
TAG=${1:-r1}
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 "$OUT/pytest_gpu.log"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 "$OUT/smoke.log"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py > "$OUT/bench.json" 2>"$OUT/bench.err"
rc=$?; echo "bench rc=$rc"; tail -c 400 "$OUT/bench.json"; echo
if [ $rc -ne 0 ]; then exit $rc; fi
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
    python3 bench.py --cpu-seconds 0 > "$OUT/prof_bench.json" 2>&1
rc=$?; echo "rocprof rc=$rc"
if [ $rc -ne 0 ]; then exit $rc; fi
bash tools/pmc_roi_pool.sh "$OUT/pmc" bench cfg2 && \
    python3 tools/summarize_pmc.py "$OUT/pmc" px8q_kernel --config cfg2 --json "$OUT/roi_pool_fwd_traffic.json" > "$OUT/pmc_summary.txt" && cat "$OUT/pmc_summary.txt"
