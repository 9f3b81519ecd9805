"""Print the A/B medians of tools/gpu_pool.sh / gpu_probe.sh logs: python tools/ab_summary.py DIR"""
import glob
import json
import os
import sys

for f in sorted(glob.glob(os.path.join(sys.argv[1], "ab_*.log"))):
    t = open(f).read()
    if "{" not in t:
        print(os.path.basename(f), "no result")
        continue
    d = json.loads(t[t.index("{"):])
    key = "variants" if "variants" in d else "paths"
    print(os.path.basename(f), d["config"], {k: round(v["us_median"], 1) for k, v in d[key].items()})
