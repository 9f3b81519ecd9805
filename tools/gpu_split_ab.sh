# A/B of the RoIPool RoI-share split inside the overlapped cfg2 bench.
set -u
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/split
mkdir -p "$OUT"
for sp in 2 3 4 2 3 4; do
  FRCNN_ROIPOOL_SPLIT=$sp timeout -k 10 120 python -u bench.py --steps 200 --warmup 20 --cpu-seconds 0 > "$OUT/b.json" 2>"$OUT/b.err"
  rc=$?; echo "split=$sp rc=$rc $(python3 -c "import json;d=json.load(open('$OUT/b.json'));print(round(d['value']), round(d['ms_per_step']*1e3,1), round(d['roofline']['kernel_us'],1))")"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
