# GPU-box script: sampler sequential-path threshold variants (FRCNN_SEQ_BELOW builds
# in tools/prev/), targets / stress parity each, cfg5 bench interleaved with the default.
set -u
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r3sb}
mkdir -p "$OUT"
for v in s1536 s2048; do
  FRCNN_LIB_PATH=$PWD/tools/prev/libfrcnn_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_targets.py tests/test_gpu_sampler_stress.py -x -q --timeout 120 --timeout-method thread > "$OUT/tests_$v.log" 2>&1; rc=$?
  echo "$v $(tail -1 $OUT/tests_$v.log)"; [ $rc -eq 0 ] || exit $rc
done
for i in 1 2; do
  for v in base s1536 s2048; do
    FRCNN_LIB_PATH=$PWD/tools/prev/libfrcnn_$v.so timeout -k 10 200 python -u bench.py --config cfg5 --cpu-seconds 0 > "$OUT/cfg5_${v}_$i.json" 2>"$OUT/cfg5_${v}_$i.err" || exit 1
    python3 -c "import json; d=json.loads(open('$OUT/cfg5_${v}_$i.json').read().strip().splitlines()[-1]); print('$v', round(d['value'],1), round(d['ms_per_step']*1000,1))"
  done
done
