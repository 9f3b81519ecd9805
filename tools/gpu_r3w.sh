set -u
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r3w}
mkdir -p "$OUT"
echo "box GPU_MAX_HW_QUEUES=${GPU_MAX_HW_QUEUES:-unset}"
run() {  # name args...
  local n=$1; shift
  timeout -k 10 200 python -u bench.py --cpu-seconds 0 "$@" > "$OUT/bench_$n.json" 2> "$OUT/bench_$n.err" || exit 1
  python3 -c "import json; s=open('$OUT/bench_$n.json').read(); d=json.loads(s[s.index('{\"metric'):].splitlines()[0]); r=d['roofline']; print('$n', round(d['value']), round(d['ms_per_step']*1e3,1), round(r['frac'],3), round(r['kernel_us_alone'],1))"
}
for i in 1 2; do
  run def_$i
  run def20_$i --steps 20 --warmup 5
  FRCNN_BENCH_HW_QUEUES=4 run q4p3_$i --prop-streams 3
done
