# cfg2 pipeline sweep: RoIPool kernel / grid size / step streams, at 300 and 20 steps.
set -u
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r3r}
mkdir -p "$OUT"
run() {  # name args...
  local n=$1; shift
  timeout -k 10 200 python -u bench.py --cpu-seconds 0 "$@" > "$OUT/bench_$n.json" 2> "$OUT/bench_$n.err" || exit 1
  python3 -c "import json; s=open('$OUT/bench_$n.json').read(); d=json.loads(s[s.index('{\"metric'):].splitlines()[0]); r=d['roofline']; print('$n', round(d['value']), round(d['ms_per_step']*1e3,1), round(r['frac'],3), round(r['kernel_us_alone'],1), r['kernel'])"
}
run pair
run w16s1 --roi-path wave --roi-split 1
run w16s1p2 --roi-path wave --roi-split 1 --prop-streams 2
run w16s1p4 --roi-path wave --roi-split 1 --prop-streams 4
run w16s2 --roi-path wave --roi-split 2
run w16s3 --roi-path wave --roi-split 3
run pair20 --steps 20 --warmup 5
run w16s1_20 --roi-path wave --roi-split 1 --steps 20 --warmup 5
run w16s2_20 --roi-path wave --roi-split 2 --steps 20 --warmup 5
run cfg1_pair --config cfg1
run cfg1_w16s1 --config cfg1 --roi-path wave --roi-split 1
