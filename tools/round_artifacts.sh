# GPU-box script: parity tests, smoke, bench lines of every BASELINE config,
# rocprofv3 kernel stats of the same bench commands, and PMC passes over the
# dominant kernels (RoIPool fwd at cfg2 / cfg4, bwd at cfg5).  Writes
# gpurun_out/$TAG; steps are chained (the first failure ends the script).
#   bash tools/round_artifacts.sh TAG
set -u
TAG=${1:-r3}
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
st() { echo "[$(date +%T)] $*"; }
st pytest
timeout -k 10 700 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
rc=$?; tail -2 "$OUT/pytest_gpu.log"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
st smoke
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || exit $?
bench() {  # name args...
  local name=$1; shift
  st "bench $name"
  timeout -k 10 300 python -u bench.py "$@" > "$OUT/bench_$name.json" 2>"$OUT/bench_$name.err" || return $?
  tail -c 300 "$OUT/bench_$name.json"; echo
}
prof() {  # name args...
  local name=$1; shift
  st "rocprof $name"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$name" -o run -- \
      python3 bench.py --cpu-seconds 0 "$@" > "$OUT/prof_$name.json" 2>&1
}
bench driver --steps 20 --warmup 5 && bench cfg2 && bench cfg1 --config cfg1 && \
bench cfg4 --config cfg4 --cpu-seconds 15 && bench cfg5 --config cfg5 && \
bench cfg3_g1 --config cfg3 --cpu-seconds 0 && bench cfg3_g2 --gpus 2 && \
prof driver --steps 20 --warmup 5 && prof cfg1 --config cfg1 && prof cfg4 --config cfg4 && \
prof cfg5 --config cfg5 && \
st "rocprof pool alone" && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
    -d "$OUT/prof_pool_alone_cfg2" -o run -- python3 tools/pool_alone.py --config cfg2 --launches 60 \
    > "$OUT/prof_pool_alone_cfg2.json" 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
    -d "$OUT/prof_pool_alone_cfg5" -o run -- python3 tools/pool_alone.py --config cfg5 --launches 60 \
    > "$OUT/prof_pool_alone_cfg5.json" 2>&1 && \
st pmc && bash tools/pmc_roi_pool.sh "$OUT/pmc_cfg2" bench cfg2 && \
bash tools/pmc_roi_pool.sh "$OUT/pmc_cfg4" bench cfg4 && \
bash tools/pmc_roi_pool.sh "$OUT/pmc_cfg5" bench cfg5
rc=$?
for c in cfg2 cfg4; do
  python3 tools/summarize_pmc.py "$OUT/pmc_$c" roi_pool_fwd_wave --config $c --json "$OUT/roi_pool_fwd_traffic.json" > "$OUT/pmc_$c.txt" 2>&1
done
python3 tools/summarize_pmc.py "$OUT/pmc_cfg5" roi_pool_bwd_lead --config cfg5 --json "$OUT/roi_pool_bwd_traffic.json" > "$OUT/pmc_cfg5.txt" 2>&1
python3 tools/summarize_pmc.py "$OUT/pmc_cfg5" roi_pool_fwd_wave --config cfg5 --json "$OUT/roi_pool_fwd_traffic.json" >> "$OUT/pmc_cfg5.txt" 2>&1
st done
exit $rc
