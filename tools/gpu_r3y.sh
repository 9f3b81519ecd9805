# Sampler: window path below 1024 steps (FRCNN_SEQ_BELOW 256 / 512) -- tests, probe, cfg5 bench.
set -u
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r3y}
mkdir -p "$OUT"
for v in 256 512; do
  FRCNN_LIB_PATH=$PWD/tools/prev/libfrcnn_seq$v.so timeout -k 10 400 python -u -m pytest tests/test_gpu_targets.py tests/test_gpu_train.py -x -q --timeout 120 --timeout-method thread > "$OUT/targets_$v.log" 2>&1; rc=$?; tail -1 "$OUT/targets_$v.log"; [ $rc -eq 0 ] || exit $rc
done
for lib in SP SP256; do
  FRCNN_LIB_PATH=$PWD/tools/prev/libfrcnn_$lib.so timeout -k 10 200 python -u tools/probe_sampler.py > "$OUT/probe_$lib.json" 2>&1 || exit 1
  grep "_targets" "$OUT/probe_$lib.json" | cut -c1-48
done
run() {  # name lib args...
  local n=$1 lib=$2; shift 2
  FRCNN_LIB_PATH=$PWD/$lib timeout -k 10 200 python -u bench.py --cpu-seconds 0 "$@" > "$OUT/bench_$n.json" 2> "$OUT/bench_$n.err" || exit 1
  python3 -c "import json; s=open('$OUT/bench_$n.json').read(); d=json.loads(s[s.index('{\"metric'):].splitlines()[0]); print('$n', round(d['value']), round(d['ms_per_step']*1e3,1))"
}
for i in 1 2; do
  run base_$i replication_faster_rcnn_amd/libfrcnn_mi355x.so --config cfg5 --steps 100 --warmup 10
  run s256_$i tools/prev/libfrcnn_seq256.so --config cfg5 --steps 100 --warmup 10
  run s512_$i tools/prev/libfrcnn_seq512.so --config cfg5 --steps 100 --warmup 10
done
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q -k "bwd" --timeout 120 --timeout-method thread > "$OUT/bwd_parity.log" 2>&1; rc=$?; tail -1 "$OUT/bwd_parity.log"; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for lib in tools/prev/libfrcnn_base.so replication_faster_rcnn_amd/libfrcnn_mi355x.so; do
    FRCNN_LIB_PATH=$PWD/$lib timeout -k 10 120 python -u tools/ab_roi_pool_bwd.py --paths auto --rounds 5 > "$OUT/bwd_$(basename $lib .so)_$i.json" 2>&1 || exit 1
    python3 -c "import json; s=open('$OUT/bwd_$(basename $lib .so)_$i.json').read(); d=json.loads(s[s.index('{'):]); print('$lib', {k: round(v['us_median'],1) for k,v in d['paths'].items()})"
  done
done
