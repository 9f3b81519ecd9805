# GPU-box script: kernel stats + SQ PMC passes of the RoIPool backward at cfg5.
set -u
TAG=${1:-bwdprof}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
    python3 bench.py --config cfg5 --streams 1 --steps 20 --warmup 3 --cpu-seconds 0 > "$OUT/prof_bench.json" 2>&1
rc=$?; echo "rocprof rc=$rc"
[ $rc -eq 0 ] || exit $rc
f=$(find "$OUT/prof" -name '*kernel_stats.csv' | head -1)
python3 - "$f" <<'PY'
import csv,sys
for r in csv.DictReader(open(sys.argv[1])):
    print(r["Name"][:80].ljust(80), r["Calls"], "%.1f us"%(float(r["AverageNs"])/1e3))
PY
bash tools/pmc_roi_pool.sh "$OUT/pmc" bench cfg5 && \
    python3 tools/summarize_pmc.py "$OUT/pmc" ${KERNEL:-roi_pool_bwd_lead} --config cfg5 --json "$OUT/roi_pool_bwd_traffic.json" > "$OUT/pmc_bwd.txt" && cat "$OUT/pmc_bwd.txt"
