# Balanced wave grid with XCD-aware ranges; pipeline variants of the cfg2 bench.
set -u
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r3m}
mkdir -p "$OUT"
export TMPDIR=/tmp
bash tools/gpu_ab.sh "$OUT" "cfg2:pair,wave,wave%8" "cfg1:wave,wave%8" || exit 1
run() {  # name args...
  local n=$1; shift
  timeout -k 10 200 python -u bench.py --steps 300 --warmup 20 --cpu-seconds 0 "$@" > "$OUT/bench_$n.json" 2> "$OUT/bench_$n.err" || exit 1
  python3 -c "import json; s=open('$OUT/bench_$n.json').read(); d=json.loads(s[s.index('{\"metric'):].splitlines()[0]); r=d['roofline']; print('$n', round(d['value']), round(d['ms_per_step']*1e3,1), round(r['frac'],3), round(r['kernel_us_alone'],1))"
}
run A
run B --pool-on own --prop-streams 2 --pool-free-cus 8
run C --pool-on own --prop-streams 3 --pool-free-cus 8
run D --pool-on own --prop-streams 2
run E --pool-free-cus 8
run F --pool-on own --prop-streams 2 --pool-free-cus 16
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/prof_B" -o run -- \
    python3 bench.py --steps 40 --warmup 5 --cpu-seconds 0 --pool-on own --prop-streams 2 --pool-free-cus 8 > "$OUT/prof_B.json" 2>&1 || exit 1
echo done
