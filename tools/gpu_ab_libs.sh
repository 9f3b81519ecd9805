# GPU-box script: RoIPool A/B across library builds (in-tree "new" and
# tools/prev/libfrcnn_<name>.so), alternating rounds, same box.
#   bash tools/gpu_ab_libs.sh TAG "cfg2 cfg4" new prev A B ...
set -u
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/$1; CFGS=$2; shift 2
mkdir -p "$OUT"
export TMPDIR=/tmp
for rnd in 1 2; do
  for c in $CFGS; do
    for lib in "$@"; do
      if [ $lib = new ]; then unset FRCNN_LIB_PATH; else export FRCNN_LIB_PATH=$PWD/tools/prev/libfrcnn_$lib.so; fi
      timeout -k 10 200 python -u tools/ab_roi_pool.py --config $c --variants wave > "$OUT/ab_${c}_${lib}_$rnd.log" 2>&1 || { tail -5 "$OUT/ab_${c}_${lib}_$rnd.log"; exit 1; }
    done
  done
done
python tools/ab_summary.py "$OUT"
