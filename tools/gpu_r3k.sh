# Balanced wave-kernel grid with interleaved RoI order: pool alone, cfg2 bench,
# kernel trace of the bench with the pool leaving 8 CUs free.
set -u
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r3k}
mkdir -p "$OUT"
export TMPDIR=/tmp
bash tools/gpu_ab.sh "$OUT" "cfg2:pair,wave,wave%8,wave%16" "cfg1:wave,wave%8" || exit 1
for k in 0 8; do
  timeout -k 10 200 python -u bench.py --steps 300 --warmup 20 --cpu-seconds 0 --pool-free-cus $k > "$OUT/bench_f$k.json" 2> "$OUT/bench_f$k.err" || exit 1
  python3 -c "import json; s=open('$OUT/bench_f$k.json').read(); d=json.loads(s[s.index('{\"metric'):].splitlines()[0]); r=d['roofline']; print('free $k', round(d['value']), round(d['ms_per_step']*1e3,1), round(r['frac'],3), round(r['kernel_us_alone'],1))"
done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/prof_f8" -o run -- \
    python3 bench.py --steps 40 --warmup 5 --cpu-seconds 0 --pool-free-cus 8 > "$OUT/prof_f8.json" 2>&1 || exit 1
