set -u
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r3b}
mkdir -p "$OUT"
export TMPDIR=/tmp
echo "[$(date +%T)] pytest"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
rc=$?; tail -3 "$OUT/pytest_gpu.log"; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_ab.sh "$OUT" cfg2:pair,wave cfg4:pair,wave cfg1:pair,wave cfg5:pair,wave || exit 1
echo "[$(date +%T)] bench"
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --cpu-seconds 0 > "$OUT/bench_driver.json" 2> "$OUT/bench_driver.err" || exit $?
tail -c 700 "$OUT/bench_driver.json"
timeout -k 10 300 python -u bench.py --cpu-seconds 0 > "$OUT/bench_300.json" 2> "$OUT/bench_300.err" || exit $?
tail -c 300 "$OUT/bench_300.json"
