# GPU-box script: parity tests of the working tree, then RoIPool A/B and cfg2
# bench of the working tree's library against tools/prev/libfrcnn_prev.so
# (a build of the previous commit), alternating, same box.
set -u
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-ablib}
mkdir -p "$OUT"
export TMPDIR=/tmp
st() { echo "[$(date +%T)] $*"; }
st pytest
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_dist.py -m gpu -x -q -k "roi_pool or dist" \
    --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
PREV=$PWD/tools/prev/libfrcnn_prev.so
for rnd in 1 2; do
  for c in cfg2 cfg4 cfg1; do
    for lib in new prev; do
      if [ $lib = prev ]; then export FRCNN_LIB_PATH=$PREV; else unset FRCNN_LIB_PATH; fi
      timeout -k 10 200 python -u tools/ab_roi_pool.py --config $c --variants wave > "$OUT/ab_${c}_${lib}_$rnd.log" 2>&1 || { tail -5 "$OUT/ab_${c}_${lib}_$rnd.log"; exit 1; }
    done
  done
done
unset FRCNN_LIB_PATH
python tools/ab_summary.py "$OUT" 2>&1 | sed 's/^/  /'
ls "$OUT"/ab_*.log | sort
for rnd in 1 2; do
  for lib in new prev; do
    if [ $lib = prev ]; then export FRCNN_LIB_PATH=$PREV; else unset FRCNN_LIB_PATH; fi
    timeout -k 10 200 python -u bench.py --cpu-seconds 0 --steps 300 > "$OUT/bench_${lib}_$rnd.json" 2>"$OUT/bench_${lib}_$rnd.err" || { tail -5 "$OUT/bench_${lib}_$rnd.err"; exit 1; }
    python - "$OUT/bench_${lib}_$rnd.json" $lib <<'PY'
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("  ", sys.argv[2], round(d["value"]), "img/s", round(d["ms_per_step"]*1e3,1), "us/step; pool", round(d["roofline"]["kernel_us"],1), "us; issue", round(d["host_issue_us_per_step"],1), "us")
PY
  done
done
if [ -n "${PROBE:-}" ]; then
  CFGS="$PROBE" bash tools/gpu_pp.sh "${1:-ablib}/pp" || exit $?
fi
