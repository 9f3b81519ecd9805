# pair vs wave RoIPool forward in the bench pipeline (cfg2 at 300 and 20 steps, cfg1), two rounds.
set -u
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r3s}
mkdir -p "$OUT"
run() {  # name args...
  local n=$1; shift
  timeout -k 10 200 python -u bench.py --cpu-seconds 0 "$@" > "$OUT/bench_$n.json" 2> "$OUT/bench_$n.err" || exit 1
  python3 -c "import json; s=open('$OUT/bench_$n.json').read(); d=json.loads(s[s.index('{\"metric'):].splitlines()[0]); r=d['roofline']; print('$n', round(d['value']), round(d['ms_per_step']*1e3,1), round(r['frac'],3), round(r['kernel_us_alone'],1), r['kernel'])"
}
for i in 1 2; do
  run pair_$i --roi-path pair
  run wave_$i --roi-path wave
  run pair20_$i --roi-path pair --steps 20 --warmup 5
  run wave20_$i --roi-path wave --steps 20 --warmup 5
  run cfg1_pair_$i --config cfg1 --roi-path pair
  run cfg1_wave_$i --config cfg1 --roi-path wave
done
