# Per-workgroup timeline of the wave forward (default vs balanced grid) and a
# kernel trace of the cfg2 bench with the latency-priority proposal kernels.
set -u
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r3l}
mkdir -p "$OUT"
export TMPDIR=/tmp
for f in 0 8; do
  FRCNN_LIB_PATH=$PWD/tools/prev/libfrcnn_PP.so timeout -k 10 120 python -u tools/probe_pool.py --config cfg2 --path wave --free $f --reps 3 > "$OUT/probe_cfg2_f$f.json" 2>&1 || exit 1
  FRCNN_LIB_PATH=$PWD/tools/prev/libfrcnn_PP.so timeout -k 10 120 python -u tools/probe_pool.py --config cfg1 --path wave --free $f --reps 3 > "$OUT/probe_cfg1_f$f.json" 2>&1 || exit 1
done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/prof_f0" -o run -- \
    python3 bench.py --steps 40 --warmup 5 --cpu-seconds 0 > "$OUT/prof_f0.json" 2>&1 || exit 1
echo done
