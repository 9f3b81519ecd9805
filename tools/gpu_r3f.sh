# A/B of the bin-row RoIPool forward vs the pair / wave kernels (bit-equality
# checked against the first variant), cfg2 / cfg1 / cfg5 shapes.
set -u
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r3f}
mkdir -p "$OUT"
bash tools/gpu_ab.sh "$OUT" cfg2:pair,row,wave cfg1:wave,row cfg5:wave,row cfg3:pair,row || exit 1
FRCNN_LIB_PATH=$PWD/tools/prev/libfrcnn_exp1.so timeout -k 10 120 python -u tools/ab_roi_pool.py --config cfg2 --variants row > "$OUT/row_nostore.json" 2>&1 || exit 1
python3 -c "import json; s=open('$OUT/row_nostore.json').read(); d=json.loads(s[s.index('{'):]); print('row no-store', {k: round(v['us_median'],1) for k,v in d['variants'].items()})"
