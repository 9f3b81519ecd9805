# GPU-box script: RoIPool backward parity + A/B (ring variants vs plain) on the cfg5 bench.
set -u
TAG=${1:-bwd}
shift || true
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_train.py tests/test_gpu_dropin.py -x -q --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 "$OUT/pytest.log"
[ $rc -eq 0 ] || exit $rc
# each arg: ENV=VAL[,ENV=VAL] ("-" = defaults)
for spec in "$@"; do
  envs=$(echo "$spec" | tr ',' ' '); [ "$spec" = "-" ] && envs=""
  env $envs timeout -k 10 200 python -u bench.py --config cfg5 --streams 1 --cpu-seconds 0 > "$OUT/bench.json" 2>&1
  rc=$?; echo "bench cfg5 [$spec] rc=$rc"
  [ $rc -eq 0 ] || exit $rc
  python3 -c "
import json
d=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1])
r=d['roofline']; print('  value %.0f img/s  bwd %.1f us (frac %.3f)  fwd %.1f us' % (d['value'], r['kernel_us'], r['frac'], r['fwd_us']))"
done
