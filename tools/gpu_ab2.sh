# GPU-box script: RoIPool parity tests of the working tree, then A/B of the
# forward kernel (working tree vs tools/prev/libfrcnn_prev.so) at cfg2/cfg4/cfg1,
# then the timeline probes (PP: with stores, PPNS: without).
set -u
cd "$GRAFT_REPO_ROOT"
T=${1:-ab2}
OUT=gpurun_out/$T
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "roi_pool" \
    --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
PREV=$PWD/tools/prev/libfrcnn_prev.so
for rnd in 1 2; do
  for c in ${CFGS:-cfg2 cfg4 cfg1}; do
    for lib in new prev; do
      if [ $lib = prev ]; then export FRCNN_LIB_PATH=$PREV; else unset FRCNN_LIB_PATH; fi
      timeout -k 10 200 python -u tools/ab_roi_pool.py --config $c --variants wave > "$OUT/ab_${c}_${lib}_$rnd.log" 2>&1 || { tail -5 "$OUT/ab_${c}_${lib}_$rnd.log"; exit 1; }
    done
  done
done
unset FRCNN_LIB_PATH
python tools/ab_summary.py "$OUT" 2>&1 | sed 's/^/  /'
CFGS="cfg2" LIB=PP bash tools/gpu_pp.sh $T/pp && CFGS="cfg2" LIB=PPNS bash tools/gpu_pp.sh $T/ppns
