# PMC passes (one rocprofv3 run each) over the draws' kernels of tools/dbg/draws_once.py
set -u
OUT=$1
mkdir -p "$OUT"
export TMPDIR=/tmp
i=0
for pmc in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_ANY SQ_INSTS_BRANCH"; do
  i=$((i + 1))
  timeout -s KILL 90 rocprofv3 --pmc $pmc --output-format csv -d "$OUT/p$i" -o run -- python3 tools/dbg/draws_once.py --reps 3 \
      > "$OUT/p$i.log" 2>&1 || { echo "pass $i failed"; tail -5 "$OUT/p$i.log"; exit 1; }
done
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(sys.argv[1] + "/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        n = r["Kernel_Name"]
        if "draw_" not in n:
            continue
        acc[n.split("(")[0][-30:]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, cs in acc.items():
    print(k)
    for c, v in sorted(cs.items()):
        print(f"   {c:24s} " + " ".join(f"{x:.3g}" for x in v[:6]))
PY
