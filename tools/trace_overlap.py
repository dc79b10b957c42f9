"""Per-kernel duration split by what overlapped it (rocprofv3 kernel trace csv).

usage: python tools/trace_overlap.py DIR KERNEL [--last N]
For each launch of KERNEL: its duration, and the names of launches on other streams that overlap
it, with the overlapped time.  Summary: mean duration alone vs overlapped.
"""
import csv
import glob
import sys
from collections import defaultdict


def load(d):
    f = glob.glob(d + "/*kernel_trace.csv")[0]
    rows = []
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"].split("(")[0].replace("tr::", "")
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name, int(r["Stream_Id"])))
    rows.sort()
    return rows


def main():
    d, k = sys.argv[1], sys.argv[2]
    last = int(sys.argv[sys.argv.index("--last") + 1]) if "--last" in sys.argv else 10 ** 9
    rows = load(d)
    mine = [r for r in rows if r[2] == k][-last:]
    alone, over = [], []
    share = defaultdict(float)
    for s, e, _, st in mine:
        ov = 0
        for s2, e2, n2, st2 in rows:
            if st2 == st or e2 <= s or s2 >= e:
                continue
            t = min(e, e2) - max(s, s2)
            ov += t
            share[n2] += t / 1e3
        (over if ov > 0.2 * (e - s) else alone).append((e - s) / 1e3)
    n = len(mine)
    print("%s: %d launches, mean %.1f us" % (k, n, sum((e - s) for s, e, _, _ in mine) / 1e3 / max(n, 1)))
    if alone:
        print("  mostly alone: %d, mean %.1f us" % (len(alone), sum(alone) / len(alone)))
    if over:
        print("  overlapped  : %d, mean %.1f us" % (len(over), sum(over) / len(over)))
    for nm, t in sorted(share.items(), key=lambda x: -x[1])[:8]:
        print("  overlap with %-18s %.1f us per launch" % (nm, t / max(n, 1)))


if __name__ == "__main__":
    main()
