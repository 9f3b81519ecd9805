# GPU-box script: persistent work-stealing RoIPool forward -- parity tests,
# kernel A/B vs tools/prev/libfrcnn_prev.so, timeline probe, and the cfg2 bench
# with the proposal streams on reserved CUs (--prop-cus K) vs shared.
set -u
cd "$GRAFT_REPO_ROOT"
T=${1:-steal}
OUT=gpurun_out/$T
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_dist.py tests/test_gpu_train.py tests/test_gpu_dropin.py -m gpu -x -q \
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
CFGS="cfg2" LIB=PP bash tools/gpu_pp.sh $T/pp || exit 1
for rnd in 1 2; do
  for k in 0 8 16 32; do
    timeout -k 10 200 python -u bench.py --cpu-seconds 0 --steps 300 --prop-cus $k > "$OUT/bench_${k}_$rnd.json" 2>"$OUT/bench_${k}_$rnd.err" || { tail -5 "$OUT/bench_${k}_$rnd.err"; exit 1; }
    python3 - "$OUT/bench_${k}_$rnd.json" "prop-cus=$k" <<'PY'
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("  ", sys.argv[2], round(d["value"]), "img/s", round(d["ms_per_step"]*1e3,1), "us/step; pool", round(d["roofline"]["kernel_us"],1), "us; issue", round(d["host_issue_us_per_step"],1))
PY
  done
done
