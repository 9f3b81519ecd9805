# Proposal-path check on the GPU: proposal / nms tests, then A/B timings of
# the wide path (cfg1, cfg4) and a kernel trace of cfg4.
set -u
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-prop}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -q --maxfail 10 --timeout 120 --timeout-method thread \
    -k "propose or nms or proposal or dropin or train or dist" > "$OUT/pytest.log" 2>&1
rc=$?; tail -3 "$OUT/pytest.log"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u tools/ab_propose.py --config cfg1 --paths wide,hybrid > "$OUT/ab_prop_cfg1.log" 2>&1 && \
timeout -k 10 200 python -u tools/ab_propose.py --config cfg4 --paths wide > "$OUT/ab_prop_cfg4.log" 2>&1 && \
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_prop4" -o run -- \
    python3 tools/ab_propose.py --config cfg4 --paths wide --rounds 2 --iters 5 > "$OUT/prof_prop4.log" 2>&1
rc=$?
grep -h -A3 '"wide"\|"hybrid"' "$OUT"/ab_prop_*.log
exit $rc
