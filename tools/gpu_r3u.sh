set -u
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r3u}
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > "$OUT/parity.log" 2>&1; rc=$?; tail -2 "$OUT/parity.log"; [ $rc -eq 0 ] || exit $rc
FRCNN_LIB_PATH=$PWD/tools/prev/libfrcnn_SP.so timeout -k 10 200 python -u tools/probe_sampler.py > "$OUT/probe_sampler.json" 2>&1 || exit 1
tail -30 "$OUT/probe_sampler.json"
