# A/B of --prop-streams on the cfg2 bench (and a dp1 cfg3-sized sanity run).
set -u
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/ps
mkdir -p "$OUT"
for ps in 1 2 3 1 2 3; do
  timeout -k 10 120 python -u bench.py --steps 200 --warmup 20 --cpu-seconds 0 --prop-streams $ps > "$OUT/b$ps.json" 2>"$OUT/b$ps.err"
  rc=$?; echo "ps=$ps rc=$rc $(python3 -c "import json;d=json.load(open('$OUT/b$ps.json'));print(round(d['value']), round(d['roofline']['kernel_us'],1))")"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
