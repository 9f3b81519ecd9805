#!/bin/bash
out=gpurun_out/cfg1sweep; mkdir -p $out
run() {
  timeout -k 10 200 python bench.py --config cfg1 --steps 100 --warmup 10 --cpu-seconds 0 "$@" > $out/b.json 2>/dev/null || { echo "FAILED $*"; return 1; }
  python3 -c "import json; d=json.loads(open('$out/b.json').read().strip().splitlines()[-1]); r=d['roofline']; print(round(d['value'],1), round(d['ms_per_step']*1e3,1), 'alone', round(r.get('kernel_us_alone') or 0,1), r.get('kernel'), '$*')"
}
run && run --roi-split 6 && run --roi-split 8 && run --roi-split 10 && run --roi-split 12 && run --roi-split 8 --roi-cg 8 && \
run --roi-split 4 --roi-cg 8 && run --roi-split 8 --roi-store nt && run --roi-split 8 && run --roi-split 6
