# A/B of two library builds on the RoIPool forward (interleaved processes):
#   bash tools/gpu_ab2.sh OUTDIR LIB_A LIB_B cfg:variants ...
set -u
cd "$GRAFT_REPO_ROOT"
OUT=$1; A=$2; B=$3; shift 3
mkdir -p "$OUT"
for i in 1 2; do
  for lib in "$A" "$B"; do
    n=$(basename "$lib" .so)
    for spec in "$@"; do
      cfg=${spec%%:*}; vars=${spec#*:}
      FRCNN_LIB_PATH=$PWD/$lib timeout -k 10 120 python -u tools/ab_roi_pool.py --config "$cfg" --variants "$vars" > "$OUT/${n}_${cfg}_$i.json" 2>&1 || { tail -3 "$OUT/${n}_${cfg}_$i.json"; exit 1; }
      python3 -c "import json; s=open('$OUT/${n}_${cfg}_$i.json').read(); d=json.loads(s[s.index('{'):]); print('$n $cfg', {k: round(v['us_median'],1) for k,v in d['variants'].items()})"
    done
  done
done
