set -u
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r3c}
mkdir -p "$OUT"
export TMPDIR=/tmp
st() { echo "[$(date +%T)] $*"; }
st bwd_ab
for i in 1 2; do
  for lib in tools/prev/libfrcnn_r3base.so replication_faster_rcnn_amd/libfrcnn_mi355x.so; do
    FRCNN_LIB_PATH=$PWD/$lib timeout -k 10 120 python -u tools/ab_roi_pool_bwd.py --paths auto --rounds 5 > "$OUT/bwd_$(basename $lib .so)_$i.json" 2>&1 || exit 1
    python3 -c "import json; s=open('$OUT/bwd_$(basename $lib .so)_$i.json').read(); d=json.loads(s[s.index('{'):]); print('$lib', {k: round(v['us_median'],1) for k,v in d['paths'].items()})"
  done
done
st bench_driver
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > "$OUT/bench_driver.json" 2> "$OUT/bench_driver.err" || exit $?
tail -c 900 "$OUT/bench_driver.json"; echo
st pmc_pair
bash tools/pmc_roi_pool.sh "$OUT/pmc_pair" pair cfg2 || exit 1
st pmc_wave
bash tools/pmc_roi_pool.sh "$OUT/pmc_wave" wave cfg2 || exit 1
st prof_driver
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_driver" -o run -- \
    python3 bench.py --steps 20 --warmup 5 --cpu-seconds 0 > "$OUT/prof_driver.json" 2>&1 || exit $?
st bench_cfg3_g1
timeout -k 10 300 python -u bench.py --config cfg3 --cpu-seconds 0 > "$OUT/bench_cfg3_g1.json" 2> "$OUT/bench_cfg3_g1.err" || exit $?
tail -c 300 "$OUT/bench_cfg3_g1.json"; echo
st done
