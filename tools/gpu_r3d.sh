set -u
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r3d}
mkdir -p "$OUT"
st() { echo "[$(date +%T)] $*"; }
pr() { python3 -c "import json,sys; s=open('$1').read(); d=json.loads(s[s.index('{'):]); k='paths' if 'paths' in d else 'variants'; print('$1'.split('/')[-1], d.get('counts',''), {p: round(v['us_median'],1) for p,v in d[k].items()})"; }
st prop_all
timeout -k 10 120 python -u tools/ab_propose.py --config cfg2 --paths hybrid,lazy > "$OUT/prop_all.json" 2>&1 || exit 1; pr "$OUT/prop_all.json"
for k in 8 16 32; do
  timeout -k 10 120 python -u tools/ab_propose.py --config cfg2 --paths hybrid,lazy --cus $k > "$OUT/prop_cus$k.json" 2>&1 || exit 1; pr "$OUT/prop_cus$k.json"
done
st pool_excl
for k in 8 16; do
  timeout -k 10 120 python -u tools/ab_roi_pool.py --config cfg2 --variants pair,pair@2,wave,wave@3 --exclude-cus $k > "$OUT/pool_ex$k.json" 2>&1 || exit 1; pr "$OUT/pool_ex$k.json"
done
timeout -k 10 120 python -u tools/ab_roi_pool.py --config cfg2 --variants pair,pair@2,wave,wave@3 > "$OUT/pool_all.json" 2>&1 || exit 1; pr "$OUT/pool_all.json"
st done
