# GPU-box script: target-assignment + training-step parity, then the cfg5 bench.
set -u
TAG=${1:-tgt}
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_targets.py tests/test_gpu_train.py -x -q --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 "$OUT/pytest.log"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u bench.py --config cfg5 --streams 1 --cpu-seconds 0 > "$OUT/bench.json" 2>&1
rc=$?; echo "bench cfg5 rc=$rc"; tail -c 700 "$OUT/bench.json"
[ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
    python3 bench.py --config cfg5 --streams 1 --steps 20 --warmup 3 --cpu-seconds 0 > "$OUT/prof_bench.json" 2>&1
rc=$?; echo "rocprof rc=$rc"
f=$(find "$OUT/prof" -name '*kernel_stats.csv' | head -1)
python3 - "$f" <<'PY'
import csv,sys
for r in list(csv.DictReader(open(sys.argv[1])))[:14]:
    print(r["Name"][:70].ljust(70), r["Calls"], "%.1f us"%(float(r["AverageNs"])/1e3))
PY
