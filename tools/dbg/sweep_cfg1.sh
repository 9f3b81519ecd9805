#!/bin/bash
# cfg1 pipeline knobs, one bench run each (100 steps): prints images/s and us/step
out=gpurun_out/cfg1sweep; mkdir -p $out
run() {
  timeout -k 10 200 python bench.py --config cfg1 --steps 100 --warmup 10 --cpu-seconds 0 "$@" > $out/b.json 2>/dev/null || { echo "FAILED $*"; return 1; }
  python3 -c "import json; d=json.loads(open('$out/b.json').read().strip().splitlines()[-1]); print(round(d['value'],1), round(d['ms_per_step']*1e3,1), '$*')"
}
run && run --prop-streams 6 && run --prop-streams 8 && run --prop-streams 3 && run --pool-on split && \
run --roi-split 4 && run --roi-split 8 && run --propose-path lazy && run --propose-path hybrid && run --prop-streams 6 --pool-on split && run
