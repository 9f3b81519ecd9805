# GPU-box script (round 2): parity tests, RoIPool forward A/B, bench lines for
# every BASELINE config, the 2-rank path, and a rocprofv3 kernel-stats run of
# the default bench.  Steps are chained: the first failure ends the script.
#   bash tools/gpu_r2.sh TAG [pytest-args...]
set -u
TAG=${1:-r2}
shift || true
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "[$(date +%T)] $name"
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "  rc=$rc"; tail -n 3 "$OUT/$name.log"
  return $rc
}
step pytest 900 python -u -m pytest tests -m gpu -q --maxfail 20 --timeout 120 --timeout-method thread "$@"
rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
step ab_cfg2 200 python -u tools/ab_roi_pool.py --config cfg2 --variants dense,dense@1,dense@3,dense@4,unsorted && \
step ab_cfg4 200 python -u tools/ab_roi_pool.py --config cfg4 --variants dense,dense@2,dense@8,unsorted && \
step ab_cfg5 200 python -u tools/ab_roi_pool.py --config cfg5 --variants dense,dense@1,dense@3,unsorted && \
step bench_cfg2 300 python -u bench.py && \
step bench_cfg1 300 python -u bench.py --config cfg1 && \
step bench_cfg4 300 python -u bench.py --config cfg4 --cpu-seconds 15 && \
step bench_cfg5 300 python -u bench.py --config cfg5 && \
step bench_cfg3_g2 300 python -u bench.py --gpus 2 && \
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && \
step prof_cfg2 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_cfg2" -o run -- \
    python3 bench.py --cpu-seconds 0 && \
step prof_cfg4 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_cfg4" -o run -- \
    python3 bench.py --config cfg4 --cpu-seconds 0
rc=$?
for f in $(find "$OUT" -name '*kernel_stats.csv'); do
  echo "== $f"; cut -d, -f1-4 "$f" | head -14
done
exit $rc
