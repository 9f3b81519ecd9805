# Sorted-forward probes (round 2, temporary): A/B incl. no-store / prep-only
# probes and a kernel trace of the same A/B run.
set -u
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-probe}
mkdir -p "$OUT"
export TMPDIR=/tmp
V=sorted,sorted!1,dense,dense!1,dense:8,dense@1,dense@4
timeout -k 10 200 python -u tools/ab_roi_pool.py --config cfg2 --variants $V > "$OUT/ab_cfg2.log" 2>&1 && \
timeout -k 10 200 python -u tools/ab_roi_pool.py --config cfg4 --variants dense,dense:8,dense:8@2,dense:8@8,dense:4 > "$OUT/ab_cfg4.log" 2>&1 && \
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
    python3 tools/ab_roi_pool.py --config cfg2 --variants sorted,dense --rounds 2 --iters 5 > "$OUT/prof.log" 2>&1
rc=$?


[ $rc -eq 0 ] && bash tools/pmc_roi_pool.sh "$OUT/pmc_dense" dense cfg2 > "$OUT/pmc_dense.log" 2>&1
rc=$?
[ $rc -eq 0 ] && bash tools/pmc_roi_pool.sh "$OUT/pmc_dense_ns" 'dense!1' cfg2 > "$OUT/pmc_dense_ns.log" 2>&1
rc=$?
cat "$OUT"/pmc_*.log

exit $rc
