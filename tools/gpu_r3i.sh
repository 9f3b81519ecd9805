# Proposal chain on k reserved CUs vs all; bench cfg2 with --prop-cus k.
set -u
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r3i}
mkdir -p "$OUT"
pr() { python3 -c "import json,sys; s=open('$1').read(); d=json.loads(s[s.index('{'):]); k='paths' if 'paths' in d else 'variants'; print('$1'.split('/')[-1], {p: round(v['us_median'],1) for p,v in d[k].items()})"; }
for k in 0 8 16 32; do
  timeout -k 10 120 python -u tools/ab_propose.py --config cfg2 --paths hybrid,lazy --cus $k > "$OUT/prop_cus$k.json" 2>&1 || exit 1; pr "$OUT/prop_cus$k.json"
done
for k in 0 16 32; do
  timeout -k 10 200 python -u bench.py --steps 300 --warmup 20 --cpu-seconds 0 --prop-cus $k > "$OUT/bench_pc$k.json" 2> "$OUT/bench_pc$k.err" || exit 1
  python3 -c "import json; s=open('$OUT/bench_pc$k.json').read(); d=json.loads(s[s.index('{\"metric'):].splitlines()[0]); print('prop_cus $k', round(d['value']), round(d['ms_per_step']*1e3,1), d['roofline']['kernel'])"
done
