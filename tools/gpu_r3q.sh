# Sampler rounds: GPU target / train tests, cfg5 bench A/B (base lib vs current).
set -u
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r3q}
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest tests/test_gpu_targets.py tests/test_gpu_train.py -x -q --timeout 120 --timeout-method thread > "$OUT/targets.log" 2>&1; rc=$?; tail -2 "$OUT/targets.log"; [ $rc -eq 0 ] || exit $rc
run() {  # name lib args...
  local n=$1 lib=$2; shift 2
  FRCNN_LIB_PATH=$PWD/$lib timeout -k 10 200 python -u bench.py --cpu-seconds 0 "$@" > "$OUT/bench_$n.json" 2> "$OUT/bench_$n.err" || exit 1
  python3 -c "import json; s=open('$OUT/bench_$n.json').read(); d=json.loads(s[s.index('{\"metric'):].splitlines()[0]); r=d['roofline']; print('$n', round(d['value']), round(d['ms_per_step']*1e3,1), round(r['frac'],3), round(r['kernel_us_alone'],1))"
}
for i in 1 2; do
  run base_cfg5_$i tools/prev/libfrcnn_base.so --config cfg5 --steps 100 --warmup 10
  run new_cfg5_$i replication_faster_rcnn_amd/libfrcnn_mi355x.so --config cfg5 --steps 100 --warmup 10
done
bash tools/gpu_r3p.sh "${1:-r3q}/p" || exit 1
