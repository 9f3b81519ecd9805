# cfg2 bench: step streams vs hardware queues (GPU_MAX_HW_QUEUES), wave kernel default.
set -u
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r3t}
mkdir -p "$OUT"
run() {  # name hwq args...
  local n=$1 q=$2; shift 2
  GPU_MAX_HW_QUEUES=$q timeout -k 10 200 python -u bench.py --cpu-seconds 0 "$@" > "$OUT/bench_$n.json" 2> "$OUT/bench_$n.err" || exit 1
  python3 -c "import json; s=open('$OUT/bench_$n.json').read(); d=json.loads(s[s.index('{\"metric'):].splitlines()[0]); r=d['roofline']; print('$n', round(d['value']), round(d['ms_per_step']*1e3,1), round(r['frac'],3), round(r['kernel_us_alone'],1), r['kernel'])"
}
run q4p3 4
run q8p3 8
run q8p4 8 --prop-streams 4
run q8p5 8 --prop-streams 5
run q8p6 8 --prop-streams 6
run q8p4_20 8 --prop-streams 4 --steps 20 --warmup 5
run q4p3_20 4 --steps 20 --warmup 5
