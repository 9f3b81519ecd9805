# GPU-box script: the round-end checks -- full GPU suite, smoke, the driver's bench command.
set -u
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r3final}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1; rc=$?
tail -2 "$OUT/pytest_gpu.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || exit $?
echo smoke ok
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > "$OUT/bench_driver.json" 2>"$OUT/bench_driver.err" || exit 1
python3 -c "import json; d=json.loads(open('$OUT/bench_driver.json').read().strip().splitlines()[-1]); print('driver', round(d['value'],1), round(d['ms_per_step']*1000,1), d['roofline']['frac'])"
