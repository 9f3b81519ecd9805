# GPU-box script: RoIPool backward tests, ring (two planes per wave) vs ring1
# (one) A/B at the training shape, cfg5 bench.
set -u
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-bw}
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_train.py -m gpu -q -k "bwd or backward or train or head_fused or cfg4" --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; tail -1 "$OUT/pytest.log"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u tools/ab_roi_pool_bwd.py --paths ring,ring1 --rounds 5 > "$OUT/ab.json" 2>&1 || exit 1
timeout -k 10 200 python -u bench.py --config cfg5 --cpu-seconds 0 > "$OUT/cfg5.json" 2> "$OUT/cfg5.err"
