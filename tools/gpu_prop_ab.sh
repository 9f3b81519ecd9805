# GPU-box script: proposal tests, fused-path phase probe, proposal A/B (working
# tree vs tools/prev/libfrcnn_prev.so) and cfg2 bench A/B.
set -u
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-propab}
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_dropin.py tests/test_gpu_train.py -m gpu -q -k "propos or rpn or train or golden or fused" --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; tail -1 "$OUT/pytest.log"; [ $rc -ne 0 ] && exit $rc
FRCNN_LIB_PATH=$PWD/tools/prev/libfrcnn_PR.so timeout -k 10 120 python -u tools/probe_propose.py --config cfg2 > "$OUT/probe.json" 2>&1 || exit 1
PREV=$PWD/tools/prev/libfrcnn_prev.so
for rnd in 1 2 3; do
  for lib in new prev; do
    if [ $lib = prev ]; then export FRCNN_LIB_PATH=$PREV; else unset FRCNN_LIB_PATH; fi
    timeout -k 10 200 python -u tools/ab_propose.py --config ${CFG:-cfg2} --paths hybrid > "$OUT/ab_${lib}_$rnd.log" 2>&1 || { tail -5 "$OUT/ab_${lib}_$rnd.log"; exit 1; }
  done
done
unset FRCNN_LIB_PATH
python tools/ab_summary.py "$OUT" 2>&1 | sed 's/^/  /'
for rnd in 1 2; do
  for lib in new prev; do
    if [ $lib = prev ]; then export FRCNN_LIB_PATH=$PREV; else unset FRCNN_LIB_PATH; fi
    timeout -k 10 200 python -u bench.py --cpu-seconds 0 --steps 300 > "$OUT/bench_${lib}_$rnd.json" 2>"$OUT/bench_${lib}_$rnd.err" || { tail -5 "$OUT/bench_${lib}_$rnd.err"; exit 1; }
    python3 - "$OUT/bench_${lib}_$rnd.json" $lib <<'PY'
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("  ", sys.argv[2], round(d["value"]), "img/s", round(d["ms_per_step"]*1e3,1), "us/step; pool", round(d["roofline"]["kernel_us"],1), "us")
PY
  done
done
