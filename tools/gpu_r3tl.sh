set -u
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r3tl}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d "$OUT/tl" -o run -- python3 bench.py --config cfg5 --cpu-seconds 0 --steps 40 > "$OUT/tl.json" 2>&1 || exit 1
python3 tools/stream_timeline.py "$OUT/tl/run_kernel_trace.csv" at_sample_kernel
