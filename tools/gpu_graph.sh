set -u
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/graph
mkdir -p "$OUT"
for a in "--graph 1" "--graph 0" "--graph 1 --steps 200"; do
  timeout -k 10 120 python -u bench.py --cpu-seconds 0 $a > "$OUT/b.json" 2>"$OUT/b.err"
  rc=$?; echo "$a rc=$rc $(python3 -c "import json;d=json.load(open('$OUT/b.json'));print(round(d['value']), round(d['ms_per_step']*1e3,1), round(d['host_issue_us_per_step'],1), round(d['roofline']['kernel_us'],1), round(d['roofline']['frac'],3))")"
  if [ $rc -ne 0 ]; then tail -20 "$OUT/b.err"; exit $rc; fi
done
