# GPU-box script: RoIPool backward paths -- parity tests, A/B timing at cfg5, cfg5 bench.
set -u
TAG=${1:-bwdab}
PATHS=${PATHS:-auto,ring}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py \
    -k "bwd or vs_oracle or golden" > "$OUT/pytest.log" 2>&1
rc=$?; tail -2 "$OUT/pytest.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python3 tools/ab_roi_pool_bwd.py --paths "$PATHS" --rounds 7 > "$OUT/ab.json" 2>&1
rc=$?; cat "$OUT/ab.json"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python3 bench.py --config cfg5 --cpu-seconds 0 > "$OUT/bench_cfg5.json" 2>&1
rc=$?; tail -1 "$OUT/bench_cfg5.json" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print(d['value'], d['ms_per_step'], r.get('kernel_us'), r.get('kernel_us_alone'), r.get('frac_alone'))"
exit $rc
