set -u
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/hostio
mkdir -p "$OUT"
for a in "--host-io 1" "--host-io 1 --steps 20 --config cfg1" "--host-io 0"; do
  timeout -k 10 180 python -u bench.py --cpu-seconds 0 $a > "$OUT/b.json" 2>"$OUT/b.err"
  rc=$?; cp "$OUT/b.json" "$OUT/b_$(echo $a | tr ' -' '__').json"
  echo "$a rc=$rc $(python3 -c "import json;d=json.load(open('$OUT/b.json'));print(round(d['value']), round(d['ms_per_step']*1e3,1), round(d['roofline']['kernel_us'],1))")"
  if [ $rc -ne 0 ]; then tail -20 "$OUT/b.err"; exit $rc; fi
done
