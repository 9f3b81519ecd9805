"""Per-stream busy / gap summary of a rocprofv3 kernel trace over the last
`--steps` occurrences of a marker kernel: which kernels each stream runs per
step and how long it idles.  python tools/stream_timeline.py trace.csv at_sample_kernel"""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
marker = sys.argv[2]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
by_q = collections.defaultdict(list)
for r in rows:
    by_q[(r["Queue_Id"], r.get("Stream_Id", ""))].append(r)
m = [r for r in rows if marker in r["Kernel_Name"]]
t0, t1 = int(m[len(m) // 3]["Start_Timestamp"]), int(m[-3]["Start_Timestamp"])
steps = sum(1 for r in m if t0 <= int(r["Start_Timestamp"]) < t1)
print(f"window {(t1 - t0) / 1e3:.1f} us over {steps} steps = {(t1 - t0) / 1e3 / steps:.1f} us/step")
for q, rs in by_q.items():
    rs = [r for r in rs if t0 <= int(r["Start_Timestamp"]) < t1]
    if not rs:
        continue
    busy = collections.Counter()
    for r in rs:
        name = r["Kernel_Name"].split("(")[0].replace("frcnn::", "").replace("void ", "")[:40]
        busy[name] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    tot = sum(busy.values())
    print(f"queue {q}: busy {tot / steps:.1f} us/step")
    for k, v in busy.most_common(8):
        print(f"    {k:40s} {v / steps:7.1f}")
