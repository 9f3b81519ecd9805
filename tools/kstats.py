"""Print a rocprofv3 kernel_stats.csv as a short table: kernel, calls, avg us, total %.

    python tools/kstats.py gpurun_out/TAG/prof_cfg2/run_kernel_stats.csv [N]
"""
import csv
import re
import sys


def short(name):
    name = re.sub(r"\(.*", "", name)
    return name.replace("void ", "").replace("frcnn::", "")[:60]


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 12
    for r in rows[:n]:
        print(f"{short(r['Name']):60s} {int(r['Calls']):6d} {float(r['AverageNs']) / 1e3:9.2f} us {float(r['Percentage']):6.2f} %")


if __name__ == "__main__":
    main()
