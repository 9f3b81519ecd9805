"""Per-call durations of the draws' kernels in a rocprofv3 kernel trace
(AnchorTarget / ProposalTarget calls alternate: even / odd)."""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
d = collections.defaultdict(list)
for r in rows:
    n = r["Kernel_Name"]
    if "draw_" in n or "sample_kernel" in n:
        d[n.split("(")[0][-34:]].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
for k, v in d.items():
    a = [x / 1e3 for x in v]
    ev, od = a[0::2], a[1::2]
    print(f"{k:36s} {len(v):4d}  even {sum(ev) / len(ev):7.1f}  odd {sum(od) / max(1, len(od)):7.1f}")
