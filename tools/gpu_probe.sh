# Round-2 probes: GPU tests, RoIPool dense no-store probe + PMC, wide-path
# proposal timings (A/B + kernel trace).  Steps chained; first failure ends it.
set -u
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-probe}
mkdir -p "$OUT"
export TMPDIR=/tmp
st() { echo "[$(date +%T)] $1"; }
st pytest; timeout -k 10 600 python -u -m pytest tests -m gpu -q --maxfail 30 --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; tail -3 "$OUT/pytest.log"; [ $rc -gt 1 ] && exit $rc
st ab_prop; true && \
timeout -k 10 200 python -u tools/ab_propose.py --config cfg4 --paths wide > "$OUT/ab_prop_cfg4.log" 2>&1 && \
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_prop4" -o run -- \
    python3 tools/ab_propose.py --config cfg4 --paths wide --rounds 2 --iters 5 > "$OUT/prof_prop4.log" 2>&1 && \
st ab_pool && timeout -k 10 200 python -u tools/ab_roi_pool.py --config cfg2 --variants wave,wave@1,wave@3,wave:8,dense > "$OUT/ab_cfg2.log" 2>&1 && \
timeout -k 10 200 python -u tools/ab_roi_pool.py --config cfg4 --variants wave,wave@1,wave@4,wave:4,dense:4 > "$OUT/ab_cfg4.log" 2>&1 && \
st pmc && bash tools/pmc_roi_pool.sh "$OUT/pmc_wave" wave cfg2 > "$OUT/pmc_wave.log" 2>&1
rc=$?
cat "$OUT"/ab_prop_*.log | grep -v amdgpu.ids
exit $rc
