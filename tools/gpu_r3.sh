# Round-3 GPU check: parity tests, smoke, the driver's bench command, the
# cfg3 strong-scaling N=1 point, and rocprofv3 kernel stats of the driver
# command.  Steps are chained; the first failure ends the script.
#   bash tools/gpu_r3.sh TAG
set -u
TAG=${1:-r3a}
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
st() { echo "[$(date +%T)] $*"; }
st pytest
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
rc=$?; tail -3 "$OUT/pytest_gpu.log"
[ $rc -eq 0 ] || exit $rc
st smoke
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || exit $?
st bench_driver
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > "$OUT/bench_driver.json" 2> "$OUT/bench_driver.err" || exit $?
tail -c 600 "$OUT/bench_driver.json"; echo
st bench_cfg3_g1
timeout -k 10 300 python -u bench.py --config cfg3 --cpu-seconds 0 > "$OUT/bench_cfg3_g1.json" 2> "$OUT/bench_cfg3_g1.err" || exit $?
tail -c 300 "$OUT/bench_cfg3_g1.json"; echo
st prof_driver
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_driver" -o run -- \
    python3 bench.py --steps 20 --warmup 5 --cpu-seconds 0 > "$OUT/prof_driver.json" 2>&1 || exit $?
st done
