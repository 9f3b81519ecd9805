# Latency-priority proposal / target kernels: bench A/B (base lib vs current), cfg2 and cfg5.
set -u
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r3o}
mkdir -p "$OUT"
run() {  # name lib args...
  local n=$1 lib=$2; shift 2
  FRCNN_LIB_PATH=$PWD/$lib timeout -k 10 200 python -u bench.py --cpu-seconds 0 "$@" > "$OUT/bench_$n.json" 2> "$OUT/bench_$n.err" || exit 1
  python3 -c "import json; s=open('$OUT/bench_$n.json').read(); d=json.loads(s[s.index('{\"metric'):].splitlines()[0]); r=d['roofline']; print('$n', round(d['value']), round(d['ms_per_step']*1e3,1), round(r['frac'],3), round(r['kernel_us_alone'],1))"
}
for i in 1 2; do
  run base_cfg5_$i tools/prev/libfrcnn_base.so --config cfg5 --steps 100 --warmup 10
  run prio_cfg5_$i replication_faster_rcnn_amd/libfrcnn_mi355x.so --config cfg5 --steps 100 --warmup 10
  run base_cfg2_$i tools/prev/libfrcnn_base.so
  run prio_cfg2_$i replication_faster_rcnn_amd/libfrcnn_mi355x.so
done
