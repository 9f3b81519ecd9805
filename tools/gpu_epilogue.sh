# GPU-box script: drop-in/epilogue parity tests, epilogue timing, rocprofv3 stats of it.
set -u
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/epi
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_dropin.py tests/test_gpu_train.py -x -v --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 "$OUT/pytest.log"
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 200 python -u tools/epilogue_bench.py > "$OUT/epilogue.jsonl" 2>&1
rc=$?; echo "epi rc=$rc"; cat "$OUT/epilogue.jsonl"
if [ $rc -ne 0 ]; then exit $rc; fi
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
    python3 tools/epilogue_bench.py > "$OUT/prof.log" 2>&1
rc=$?; echo "rocprof rc=$rc"
f=$(find "$OUT/prof" -name '*kernel_stats.csv' | head -1)
[ -n "$f" ] && cut -d, -f1-8 "$f" | head -20
exit $rc
