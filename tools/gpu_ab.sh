# A/B of RoIPool forward paths: bash tools/gpu_ab.sh OUTDIR cfg:variants [cfg:variants ...]
# e.g. bash tools/gpu_ab.sh gpurun_out/ab cfg2:pair,wave cfg4:pair,wave
set -u
cd "$GRAFT_REPO_ROOT"
OUT=$1; shift
mkdir -p "$OUT"
for spec in "$@"; do
  cfg=${spec%%:*}; vars=${spec#*:}
  echo "[$(date +%T)] ab $cfg $vars"
  timeout -k 10 240 python -u tools/ab_roi_pool.py --config "$cfg" --variants "$vars" > "$OUT/ab_$cfg.json" 2>&1 || { tail -5 "$OUT/ab_$cfg.json"; exit 1; }
  python3 -c "import json; s=open('$OUT/ab_$cfg.json').read(); d=json.loads(s[s.index('{'):]); print('$cfg', {k: round(v['us_median'],1) for k,v in d['variants'].items()})"
done
