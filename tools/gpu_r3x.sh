# Sampler guesses: target / train tests, sampler probe, cfg5 bench; bench HW-queue check.
set -u
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r3x}
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest tests/test_gpu_targets.py tests/test_gpu_train.py -x -q --timeout 120 --timeout-method thread > "$OUT/targets.log" 2>&1; rc=$?; tail -2 "$OUT/targets.log"; [ $rc -eq 0 ] || exit $rc
FRCNN_LIB_PATH=$PWD/tools/prev/libfrcnn_SP.so timeout -k 10 200 python -u tools/probe_sampler.py > "$OUT/probe_sampler.json" 2>&1 || exit 1
grep anchor_targets "$OUT/probe_sampler.json" | tail -1 | cut -c1-60; grep -o "cyc/window.*" "$OUT/probe_sampler.json" | head -3
run() {  # name args...
  local n=$1; shift
  timeout -k 10 200 python -u bench.py --cpu-seconds 0 "$@" > "$OUT/bench_$n.json" 2> "$OUT/bench_$n.err" || exit 1
  python3 -c "import json; s=open('$OUT/bench_$n.json').read(); d=json.loads(s[s.index('{\"metric'):].splitlines()[0]); r=d['roofline']; print('$n', round(d['value']), round(d['ms_per_step']*1e3,1), round(r['frac'],3), round(r['kernel_us_alone'],1))"
}
run cfg5 --config cfg5 --steps 100 --warmup 10
run def --steps 50


