# GPU-box script: RoIPool backward timing probes (prebuilt libs under tools/prev).
set -u
TAG=${1:-bwdprobe}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
for L in ${LIBS:-P1 P2 P3 D4}; do
    FRCNN_LIB_PATH=$PWD/tools/prev/libfrcnn_$L.so timeout -k 10 120 python3 tools/ab_roi_pool_bwd.py --paths auto --rounds 5 > "$OUT/ab_$L.json" 2>&1
    rc=$?; echo "$L $(grep us_median "$OUT/ab_$L.json")"; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 120 python3 tools/ab_roi_pool_bwd.py --paths auto,grp_rmw,ring --rounds 5 > "$OUT/ab_cur.json" 2>&1
rc=$?; echo "cur $(grep us_median "$OUT/ab_cur.json" | tr -d '\n')"; exit $rc
