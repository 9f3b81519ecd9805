set -u
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r3n}
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > "$OUT/parity.log" 2>&1; rc=$?; tail -2 "$OUT/parity.log"; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_ab2.sh "$OUT" tools/prev/libfrcnn_base.so replication_faster_rcnn_amd/libfrcnn_mi355x.so cfg2:pair,wave cfg4:wave || exit 1
bash tools/gpu_ab2.sh "$OUT/pf" replication_faster_rcnn_amd/libfrcnn_mi355x.so tools/prev/libfrcnn_pf.so cfg2:pair || exit 1
