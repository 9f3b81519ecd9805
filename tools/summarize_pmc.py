"""Summarize rocprofv3 PMC passes of tools/pmc_roi_pool.sh for one kernel.

    python tools/summarize_pmc.py <dir> <kernel-substring> [--config cfg2 --json out.json]

Per-dispatch values (averaged over dispatches), and the HBM traffic per launch
= FETCH_SIZE x 2 (gfx950 counts half of wide coalesced reads, MI355X_MICROARCH.md
§HBM) + WRITE_SIZE, both in KiB -> bytes.
"""
import argparse
import collections
import csv
import json
import os


def load(d, kern):
    out = {}
    for grp in sorted(os.listdir(d)):
        f = os.path.join(d, grp, "run_counter_collection.csv")
        if not os.path.exists(f):
            continue
        agg, disp = collections.defaultdict(float), set()
        for r in csv.DictReader(open(f)):
            if kern not in r["Kernel_Name"]:
                continue
            agg[r["Counter_Name"]] += float(r["Counter_Value"])
            disp.add(r["Dispatch_Id"])
        for k, v in agg.items():
            out[k] = v / max(len(disp), 1)
    return out


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("kernel")
    ap.add_argument("--config", default="cfg2")
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    c = load(a.dir, a.kernel)
    for k in sorted(c):
        print(f"{k:28s} {c[k]:.6g}")
    if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
        fetch = c["FETCH_SIZE"] * 2 * 1024
        write = c["WRITE_SIZE"] * 1024
        tot = fetch + write
        print(f"HBM bytes per launch: fetch(x2) {fetch:.4g} + write {write:.4g} = {tot:.4g}")
        if a.json:
            data = json.load(open(a.json)) if os.path.exists(a.json) else {}
            data[a.config] = {"kernel": a.kernel, "hbm_bytes_per_launch": tot,
                              "fetch_bytes_x2": fetch, "write_bytes": write,
                              "counters": c, "source": os.path.basename(os.path.normpath(a.dir))}
            json.dump(data, open(a.json, "w"), indent=1)
