# cfg2 bench: LDS the wave RoIPool leaves per CU (for the IoU-tile kernel) x runs.
set -u
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r3v}
mkdir -p "$OUT"
run() {  # name args...
  local n=$1; shift
  timeout -k 10 200 python -u bench.py --cpu-seconds 0 "$@" > "$OUT/bench_$n.json" 2> "$OUT/bench_$n.err" || exit 1
  python3 -c "import json; s=open('$OUT/bench_$n.json').read(); d=json.loads(s[s.index('{\"metric'):].splitlines()[0]); r=d['roofline']; print('$n', round(d['value']), round(d['ms_per_step']*1e3,1), round(r['frac'],3), round(r['kernel_us_alone'],1))"
}
for i in 1 2; do
  run l0_$i
  run l4k_$i --roi-lds-leave 4096
  run l8k_$i --roi-lds-leave 8192
  run l0_20_$i --steps 20 --warmup 5
  run l4k_20_$i --roi-lds-leave 4096 --steps 20 --warmup 5
done
