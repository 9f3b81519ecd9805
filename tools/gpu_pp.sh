# GPU-box script: RoIPool forward timeline probe (-DFRCNN_POOL_PROF build in
# tools/prev/libfrcnn_PP.so) at cfg2/cfg4/cfg5, then the product kernel alone.
set -u
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-pp}
mkdir -p "$OUT"
export FRCNN_LIB_PATH=$PWD/tools/prev/libfrcnn_${LIB:-PP}.so
for c in ${CFGS:-cfg2 cfg4 cfg5}; do
  timeout -k 10 120 python -u tools/probe_pool.py --config $c --reps 3 > "$OUT/probe_$c.json" 2>"$OUT/probe_$c.err" || exit $?
done
unset FRCNN_LIB_PATH
timeout -k 10 120 python -u tools/ab_roi_pool.py --config cfg2 --variants ${AB:-wave} > "$OUT/ab_cfg2.json" 2>&1
