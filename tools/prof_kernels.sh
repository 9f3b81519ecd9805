# rocprofv3 kernel-trace summary of one bench run (no PMC).
set -u
cd "$GRAFT_REPO_ROOT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=${1:-gpurun_out/prof}
shift || true
mkdir -p "$OUT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT" -o run -- \
    python3 bench.py --steps 20 --warmup 5 --cpu-seconds 0 "$@" > "$OUT/bench.log" 2>&1
rc=$?
echo "rc=$rc"
find "$OUT" -name '*kernel_stats.csv' | head -3
f=$(find "$OUT" -name '*kernel_stats.csv' | head -1)
[ -n "$f" ] && cut -d, -f1-8 "$f" | head -30
exit $rc
