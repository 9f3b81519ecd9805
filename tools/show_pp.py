"""Summarise tools/probe_pool.py outputs: python tools/show_pp.py gpurun_out/pp"""
import glob
import json
import sys

for f in sorted(glob.glob(sys.argv[1] + "/probe_*.json")):
    d = json.load(open(f))
    for r in d["runs"][-2:]:
        print(d["config"], "events", round(r["events_us"], 1), "span", r["span_us"], "wgs", r["wgs"],
              r["live_wgs"], "rois/wg", r["rois_per_wg"])
        for k, v in r["phases"].items():
            print("   %-8s" % k, v)
