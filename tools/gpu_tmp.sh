set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for o in 0 1; do
timeout -k 10 120 python bench.py --cpu-seconds 0 --steps 200 --order $o > gpurun_out/bo$o.json || exit 1
python3 -c "
import json; d=json.load(open('gpurun_out/bo$o.json')); print('order', $o, d['value'], d['ms_per_step'], d['roofline']['kernel_us'])"
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/po$o -o run -- python3 bench.py --cpu-seconds 0 --order $o > gpurun_out/po$o.json 2>&1 || exit 1
python3 -c "
import csv,glob
f=glob.glob('gpurun_out/po$o/**/run_kernel_stats.csv', recursive=True)[0]
for r in csv.DictReader(open(f)):
    print(r['Name'][:50], r['Calls'], r['AverageNs'])" | head -6
done
