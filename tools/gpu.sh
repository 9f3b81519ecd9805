# GPU-box driver for every measurement of the round (replaces the one-off
# tools/gpu_r3*.sh scripts): each argument after OUT is one step, run in order
# under its own time limit; the first failing step ends the script.
#   bash tools/gpu.sh gpurun_out/TAG "test -k roi_pool" "ab cfg2 key,wave" "bench driver --steps 20 --warmup 5"
# steps:
#   test [pytest args]         pytest -m gpu (all GPU tests when no args)
#   smoke                      __graft_entry__.smoke()
#   ab CFG VARIANTS [ARGS]     tools/ab_roi_pool.py (RoIPool forward paths, interleaved rounds)
#   bench NAME [bench args]    bench.py -> OUT/bench_NAME.json
#   prof NAME [bench args]     rocprofv3 --kernel-trace --stats of bench.py -> OUT/prof_NAME
#   alone CFG [LAUNCHES]       rocprofv3 of tools/pool_alone.py -> OUT/prof_alone_CFG
#   pmc CFG KERNEL             PMC passes of tools/pmc_roi_pool.sh over bench CFG, summarised for KERNEL
#   py NAME SCRIPT [args]      any python tool -> OUT/NAME.log
set -u
cd "$GRAFT_REPO_ROOT"
OUT=$1; shift
mkdir -p "$OUT"
export TMPDIR=/tmp
st() { echo "[$(date +%T)] $*"; }
run_step() {
  local kind=$1; shift
  case $kind in
    test)  # a '%' in an argument stands for a space (-k roi_pool%or%cfg5)
      local targs=("${@//%/ }")
      timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread "${targs[@]}" \
          > "$OUT/pytest_gpu.log" 2>&1; local rc=$?; tail -3 "$OUT/pytest_gpu.log"; return $rc ;;
    smoke)
      timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 ;;
    ab)
      local cfg=$1 vars=$2; shift 2
      timeout -k 10 300 python -u tools/ab_roi_pool.py --config "$cfg" --variants "$vars" "$@" \
          > "$OUT/ab_$cfg.json" 2>&1 || { tail -5 "$OUT/ab_$cfg.json"; return 1; }
      python3 -c "import json; s=open('$OUT/ab_$cfg.json').read(); d=json.loads(s[s.index('{'):]); print('$cfg', {k: round(v['us_median'],1) for k,v in d['variants'].items()})" ;;
    bench)
      local name=$1; shift
      timeout -k 10 400 python -u bench.py "$@" > "$OUT/bench_$name.json" 2>"$OUT/bench_$name.err" || { tail -5 "$OUT/bench_$name.err"; return 1; }
      python3 -c "import json; d=json.loads(open('$OUT/bench_$name.json').read().strip().splitlines()[-1]); r=d['roofline']; f=lambda v: None if v is None else round(v,3); print('$name', round(d['value'],1), 'img/s', round(d['ms_per_step']*1e3,1), 'us/step', r.get('kernel'), 'achieved', f(r.get('achieved')), 'frac', f(r.get('frac')), 'alone', f(r.get('kernel_us_alone')), f(r.get('frac_alone')))" ;;
    prof)
      local name=$1; shift
      timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$name" -o run -- \
          python3 bench.py --cpu-seconds 0 "$@" > "$OUT/prof_$name.json" 2>&1 ;;
    alone)
      local cfg=$1 n=${2:-60}
      timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_alone_$cfg" -o run -- \
          python3 tools/pool_alone.py --config "$cfg" --launches "$n" > "$OUT/prof_alone_$cfg.json" 2>&1 || return 1
      tail -c 400 "$OUT/prof_alone_$cfg.json"; echo ;;
    pmc)
      local cfg=$1 kern=$2
      bash tools/pmc_roi_pool.sh "$OUT/pmc_$cfg" bench "$cfg" || return 1
      python3 tools/summarize_pmc.py "$OUT/pmc_$cfg" "$kern" --config "$cfg" --json "$OUT/traffic_$cfg.json" \
          > "$OUT/pmc_$cfg.txt" 2>&1; cat "$OUT/pmc_$cfg.txt" ;;
    py)
      local name=$1; shift
      timeout -k 10 400 python -u "$@" > "$OUT/$name.log" 2>&1; local rc=$?; tail -20 "$OUT/$name.log"; return $rc ;;
    *) echo "unknown step $kind"; return 2 ;;
  esac
}
for step in "$@"; do
  st "$step"
  # shellcheck disable=SC2086
  run_step $step || { st "FAILED: $step"; exit 1; }
done
st done
