# cfg2 bench: RoIPool forward variants under the three-stream pipeline.
set -u
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r3p}
mkdir -p "$OUT"
run() {  # name args...
  local n=$1; shift
  timeout -k 10 200 python -u bench.py --cpu-seconds 0 "$@" > "$OUT/bench_$n.json" 2> "$OUT/bench_$n.err" || exit 1
  python3 -c "import json; s=open('$OUT/bench_$n.json').read(); d=json.loads(s[s.index('{\"metric'):].splitlines()[0]); r=d['roofline']; print('$n', round(d['value']), round(d['ms_per_step']*1e3,1), round(r['frac'],3), round(r['kernel_us_alone'],1), r['kernel'])"
}
run pair
run wave16 --roi-path wave
run wave8 --roi-path wave --roi-cg 8
run wave8s1 --roi-path wave --roi-cg 8 --roi-split 1
run wave16s1 --roi-path wave --roi-split 1
run lazy --propose-path lazy
