# GPU-box script: bench A/B over environment settings.  Args: CONFIG then specs
# "ENV=VAL[,ENV=VAL]" ("-" = defaults); extra bench flags via BENCH_FLAGS.
set -u
cd "$GRAFT_REPO_ROOT"
CFG=$1; shift
OUT=gpurun_out/envab
mkdir -p "$OUT"
for spec in "$@"; do
  envs=$(echo "$spec" | tr ',' ' '); [ "$spec" = "-" ] && envs=""
  env $envs timeout -k 10 200 python -u bench.py --config $CFG --cpu-seconds 0 ${BENCH_FLAGS:-} > "$OUT/b.json" 2>&1
  rc=$?; echo "[$spec] rc=$rc"
  [ $rc -eq 0 ] || { tail -5 "$OUT/b.json"; exit $rc; }
  python3 -c "
import json
d=json.loads(open('$OUT/b.json').read().strip().splitlines()[-1])
r=d['roofline']; print('  value %.0f img/s  ms/step %.4f  kernel %.1f us (frac %.3f)' % (d['value'], d['ms_per_step'], r['kernel_us'], r['frac']))"
done
