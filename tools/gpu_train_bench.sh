# GPU-box script: training-step (cfg5) bench + rocprofv3 kernel stats + PMC of
# the RoIPool backward; quick cfg2 bench re-check.  Writes gpurun_out/$TAG.
set -u
TAG=${1:-train}
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_targets.py tests/test_gpu_train.py -x -q --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 "$OUT/pytest.log"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u bench.py --cpu-seconds 0 > "$OUT/bench_cfg2.json" 2>"$OUT/bench_cfg2.err"
rc=$?; echo "bench cfg2 rc=$rc"; tail -c 300 "$OUT/bench_cfg2.json"; echo
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --config cfg5 --cpu-seconds 15 > "$OUT/bench_cfg5.json" 2>"$OUT/bench_cfg5.err"
rc=$?; echo "bench cfg5 rc=$rc"; cat "$OUT/bench_cfg5.json"; tail -3 "$OUT/bench_cfg5.err"; echo
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u bench.py --config cfg5 --streams 1 --cpu-seconds 0 > "$OUT/bench_cfg5_s1.json" 2>&1
rc=$?; echo "bench cfg5 s1 rc=$rc"; tail -c 400 "$OUT/bench_cfg5_s1.json"; echo
[ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
    python3 bench.py --config cfg5 --cpu-seconds 0 > "$OUT/prof_bench.json" 2>&1
rc=$?; echo "rocprof rc=$rc"
[ $rc -eq 0 ] || exit $rc
bash tools/pmc_roi_pool.sh "$OUT/pmc" bench cfg5 && \
    python3 tools/summarize_pmc.py "$OUT/pmc" roi_pool_bwd_pf --config cfg5 --json "$OUT/roi_pool_bwd_traffic.json" > "$OUT/pmc_bwd.txt" && \
    python3 tools/summarize_pmc.py "$OUT/pmc" px8q_kernel --config cfg5 --json "$OUT/roi_pool_fwd_traffic.json" > "$OUT/pmc_fwd.txt" && \
    cat "$OUT/pmc_bwd.txt" "$OUT/pmc_fwd.txt"
