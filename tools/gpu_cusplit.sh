# GPU-box script: cfg2 bench with the proposal stream on a CU partition (A/B).
set -u
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/cusplit
mkdir -p "$OUT"
for k in "$@"; do
  timeout -k 10 200 python -u bench.py --cpu-seconds 0 --prop-cus $k > "$OUT/b$k.json" 2>&1
  rc=$?; echo "prop-cus $k rc=$rc"
  [ $rc -eq 0 ] || { tail -5 "$OUT/b$k.json"; exit $rc; }
  python3 -c "
import json
d=json.loads(open('$OUT/b$k.json').read().strip().splitlines()[-1])
r=d['roofline']; print('  value %.0f img/s  ms/step %.4f  pool %.1f us (frac %.3f)' % (d['value'], d['ms_per_step'], r['kernel_us'], r['frac']))"
done
