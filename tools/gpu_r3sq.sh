# GPU-box script: sampler micro-optimisations -- targets / train / stress parity, then
# cfg5 bench interleaved with the previous library (tools/prev/libfrcnn_base.so).
set -u
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r3sq}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_targets.py tests/test_gpu_train.py tests/test_gpu_sampler_stress.py -x -q --timeout 120 --timeout-method thread > "$OUT/tests.log" 2>&1; rc=$?
tail -2 "$OUT/tests.log"; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for lib in tools/prev/libfrcnn_base.so replication_faster_rcnn_amd/libfrcnn_mi355x.so; do
    n=$(basename $lib .so)_$i
    FRCNN_LIB_PATH=$PWD/$lib timeout -k 10 200 python -u bench.py --config cfg5 --cpu-seconds 0 > "$OUT/cfg5_$n.json" 2>"$OUT/cfg5_$n.err" || exit 1
    python3 -c "import json; d=json.loads(open('$OUT/cfg5_$n.json').read().strip().splitlines()[-1]); print('$n', round(d['value'],1), round(d['ms_per_step']*1000,1))"
  done
done
FRCNN_LIB_PATH=$PWD/tools/prev/libfrcnn_SP.so timeout -k 10 200 python -u tools/probe_sampler.py > "$OUT/probe.log" 2>&1 || exit 1
cut -c1-60 "$OUT/probe.log"
timeout -k 10 200 python -u bench.py --config cfg5 > "$OUT/bench_cfg5.json" 2>"$OUT/bench_cfg5.err" || exit 1
tail -c 200 "$OUT/bench_cfg5.json"; echo
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_cfg5" -o run -- \
    python3 bench.py --cpu-seconds 0 --config cfg5 > "$OUT/prof_cfg5.json" 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d "$OUT/tl" -o run -- python3 bench.py --config cfg5 --cpu-seconds 0 --steps 40 > "$OUT/tl.json" 2>&1 || exit 1
python3 tools/stream_timeline.py "$OUT/tl/run_kernel_trace.csv" at_sample_kernel > "$OUT/timeline_cfg5.txt"
cat "$OUT/timeline_cfg5.txt"
