"""Print a kernel timeline from a rocprofv3 kernel trace (csv):

    python tools/timeline.py TRACE.csv [--first N] [--last N] [--filter SUBSTR]

One line per dispatch: start / end relative to the first printed dispatch (us),
duration, queue / stream, short kernel name.  Used to read how the bench's
step streams overlap."""
import argparse
import csv


def short(name):
    n = name.split("(")[0]
    n = n.replace("frcnn::", "")
    return n[:60]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--first", type=int, default=0, help="skip this many dispatches")
    ap.add_argument("--count", type=int, default=80)
    ap.add_argument("--filter", default="")
    a = ap.parse_args()
    rows = [r for r in csv.DictReader(open(a.trace)) if a.filter in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    rows = rows[a.first:a.first + a.count]
    if not rows:
        return
    t0 = int(rows[0]["Start_Timestamp"])
    for r in rows:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        print(f"{(s - t0) / 1e3:9.1f} {(e - t0) / 1e3:9.1f} {(e - s) / 1e3:7.1f}  q{r['Queue_Id']:>2} s{r['Stream_Id']:>2}  "
              f"{short(r['Kernel_Name'])}")


if __name__ == "__main__":
    main()
