# RoIPool forward check: pool tests, A/B at cfg2 / cfg4 / cfg5, optional PMC.
#   bash tools/gpu_pool.sh TAG [VARIANTS] [pmc]
set -u
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-pool}
V=${2:-wave,dense}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -q --maxfail 10 --timeout 120 --timeout-method thread \
    -k "roi_pool or head or golden or train" > "$OUT/pytest.log" 2>&1
rc=$?; tail -2 "$OUT/pytest.log"; [ $rc -ne 0 ] && exit $rc
for c in cfg2 cfg4 cfg5; do
  timeout -k 10 200 python -u tools/ab_roi_pool.py --config $c --variants "$V" > "$OUT/ab_$c.log" 2>&1 || exit $?
done
timeout -k 10 200 python -u tools/ab_roi_pool_bwd.py > "$OUT/ab_bwd.log" 2>&1 || exit $?
timeout -k 10 300 python -u bench.py > "$OUT/bench_cfg2.log" 2>&1 || exit $?
if [ "${3:-}" = pmc ]; then
  bash tools/pmc_roi_pool.sh "$OUT/pmc" "${V%%,*}" cfg2 > "$OUT/pmc.log" 2>&1 || exit $?
fi
exit 0
