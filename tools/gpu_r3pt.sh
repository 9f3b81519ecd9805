# GPU-box script: ProposalTarget prepare/sample split -- targets / train parity, cfg5 bench x3.
set -u
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r3pt}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_targets.py tests/test_gpu_train.py tests/test_gpu_sampler_stress.py -x -q --timeout 120 --timeout-method thread > "$OUT/tests.log" 2>&1; rc=$?
tail -2 "$OUT/tests.log"; [ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do
  timeout -k 10 200 python -u bench.py --config cfg5 --cpu-seconds 0 > "$OUT/cfg5_$i.json" 2>"$OUT/cfg5_$i.err" || exit 1
  python3 -c "import json; d=json.loads(open('$OUT/cfg5_$i.json').read().strip().splitlines()[-1]); print('cfg5', round(d['value'],1), round(d['ms_per_step']*1000,1))"
done
