# Decomposition of the RoIPool forward (no stores / no scan builds), VALU issue
# rate probe, counter list, and the CU-reservation A/B of the proposal chain.
set -u
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r3e}
mkdir -p "$OUT"
export TMPDIR=/tmp
st() { echo "[$(date +%T)] $*"; }
pr() { python3 -c "import json,sys; s=open('$1').read(); d=json.loads(s[s.index('{'):]); k='paths' if 'paths' in d else 'variants'; print('$1'.split('/')[-1], {p: round(v['us_median'],1) for p,v in d[k].items()})"; }
st valu_rate
timeout -k 10 60 tools/prev/valu_rate > "$OUT/valu_rate.txt" 2>&1 || exit 1; cat "$OUT/valu_rate.txt"
timeout -k 10 60 rocprofv3 -L > "$OUT/counters.txt" 2>&1; echo "counters rc=$?"
for lib in replication_faster_rcnn_amd/libfrcnn_mi355x.so tools/prev/libfrcnn_exp1.so tools/prev/libfrcnn_exp2.so; do
  n=$(basename $lib .so)
  FRCNN_LIB_PATH=$PWD/$lib timeout -k 10 120 python -u tools/ab_roi_pool.py --config cfg2 --variants pair,wave > "$OUT/pool_$n.json" 2>&1 || exit 1; pr "$OUT/pool_$n.json"
done
bash tools/gpu_r3d.sh "${1:-r3e}/d" || exit 1
st done
