set -u
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/issue
mkdir -p "$OUT"
for a in "--prop-streams 2" "--prop-streams 1" "--streams 1"; do
  timeout -k 10 120 python -u bench.py --steps 200 --warmup 20 --cpu-seconds 0 $a > "$OUT/b.json" 2>"$OUT/b.err"
  rc=$?; echo "$a rc=$rc $(python3 -c "import json;d=json.load(open('$OUT/b.json'));print(round(d['value']), round(d['ms_per_step']*1e3,1), round(d['host_issue_us_per_step'],1))")"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
