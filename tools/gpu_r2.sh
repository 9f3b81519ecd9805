# GPU-box script (round 2): parity tests, RoIPool forward A/B, bench lines for
# every BASELINE config, the 2-rank path, and rocprofv3 kernel-stats runs.
# Steps are chained: the first failure (other than pytest's rc=1) ends the script.
#   bash tools/gpu_r2.sh TAG STEP[,STEP...] [pytest-args...]
# STEP names: pytest ab_cfg2 ab_cfg4 ab_cfg5 bench_cfg1 bench_cfg2 bench_cfg4
#             bench_cfg5 bench_cfg3_g2 prof_cfg2 prof_cfg4 prof_cfg5
set -u
TAG=${1:-r2}
STEPS=${2:-pytest,bench_cfg2}
shift 2 || true
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "[$(date +%T)] $name"
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "  rc=$rc"; tail -n 3 "$OUT/$name.log"
  return $rc
}
prof() {  # name timeout bench-args...
  local name=$1 t=$2; shift 2
  step "$name" "$t" rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/$name" -o run -- \
      python3 bench.py --cpu-seconds 0 "$@"
}
rc=0
for s in ${STEPS//,/ }; do
  case $s in
    pytest) step pytest 900 python -u -m pytest tests -m gpu -q --maxfail 20 --timeout 120 \
              --timeout-method thread "$@"; rc=$?; [ $rc -eq 1 ] && rc=0 ;;
    ab_cfg2) step ab_cfg2 200 python -u tools/ab_roi_pool.py --config cfg2 --variants ${AB2:-sorted,sorted:8,sorted@1,sorted@4,sorted:8@4,sorted/u,dense}; rc=$? ;;
    ab_cfg4) step ab_cfg4 200 python -u tools/ab_roi_pool.py --config cfg4 --variants ${AB4:-sorted,sorted:4,sorted@2,sorted@8,sorted/u,dense}; rc=$? ;;
    ab_cfg5) step ab_cfg5 200 python -u tools/ab_roi_pool.py --config cfg5 --variants ${AB5:-sorted,sorted:8,sorted@2,sorted:8@2,dense}; rc=$? ;;
    bench_cfg1) step bench_cfg1 300 python -u bench.py --config cfg1; rc=$? ;;
    bench_cfg2) step bench_cfg2 300 python -u bench.py; rc=$? ;;
    bench_cfg4) step bench_cfg4 300 python -u bench.py --config cfg4 --cpu-seconds 15; rc=$? ;;
    bench_cfg5) step bench_cfg5 300 python -u bench.py --config cfg5; rc=$? ;;
    bench_cfg3_g2) step bench_cfg3_g2 300 python -u bench.py --gpus 2; rc=$? ;;
    prof_cfg2) prof prof_cfg2 300; rc=$? ;;
    prof_cfg4) prof prof_cfg4 300 --config cfg4; rc=$? ;;
    prof_cfg5) prof prof_cfg5 300 --config cfg5; rc=$? ;;
    *) echo "unknown step $s"; rc=2 ;;
  esac
  [ $rc -ne 0 ] && break
done
for f in $(find "$OUT" -name '*kernel_stats.csv'); do
  echo "== $f"; cut -d, -f1-4 "$f" | head -14
done
exit $rc
