# GPU-box script: cfg2 bench under RoIPool tile choices -- the default 16-channel
# tile (one workgroup per CU, all of its LDS) vs 8- and 4-channel tiles with one
# share per (image, channel group), which leave LDS and wave slots free for the
# next step's proposal kernels beside the pool.  Alternating rounds.
set -u
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-cg}
mkdir -p "$OUT"
for rnd in 1 2; do
  for v in ${VARIANTS:-auto:auto 8:1 8:2 4:1}; do
    cg=${v%%:*}; sp=${v##*:}
    timeout -k 10 200 python -u bench.py --cpu-seconds 0 --steps 300 --roi-cg $cg --roi-split $sp ${EXTRA:-} > "$OUT/bench_${cg}_${sp}_$rnd.json" 2>"$OUT/bench_${cg}_${sp}_$rnd.err" || { tail -5 "$OUT/bench_${cg}_${sp}_$rnd.err"; exit 1; }
    python3 - "$OUT/bench_${cg}_${sp}_$rnd.json" "cg=$cg split=$sp" <<'PY'
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("  ", sys.argv[2], round(d["value"]), "img/s", round(d["ms_per_step"]*1e3,1), "us/step; pool", round(d["roofline"]["kernel_us"],1), "us")
PY
  done
done
