# GPU-box script: RoIPool backward parity + A/B (ring vs plain) on the cfg5 bench.
set -u
TAG=${1:-bwd}
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_train.py tests/test_gpu_dropin.py -x -q --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 "$OUT/pytest.log"
[ $rc -eq 0 ] || exit $rc
for v in ring plain; do
  FRCNN_BWD_VARIANT=$v timeout -k 10 200 python -u bench.py --config cfg5 --streams 1 --cpu-seconds 0 > "$OUT/bench_cfg5_$v.json" 2>&1
  rc=$?; echo "bench cfg5 $v rc=$rc"; python3 -c "
import json,sys
d=json.loads(open('$OUT/bench_cfg5_$v.json').read().strip().splitlines()[-1])
print(d['value'], d['roofline'])" || exit 1
  [ $rc -eq 0 ] || exit $rc
done
