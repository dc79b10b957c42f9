"""Summarise rocprofv3 CSV output (kernel trace + PMC passes) into a markdown table.

usage: python tools/prof_summary.py TRACE_DIR [PMC_DIR ...] > profiles/<name>.md
Per kernel: launches, mean/min/max duration; for k_nn_partial the full-tree sweeps (grid.y > 8)
and the delta sweeps are listed separately.  PMC values are per launch (FETCH_SIZE / WRITE_SIZE in
KB as rocprofv3 reports them; on gfx950 FETCH_SIZE under-reports wide streaming reads by 2x)."""
import csv
import glob
import os
import sys
from collections import defaultdict


def short(name):
    return name.split("(")[0].replace("tr::", "")


def key(r):
    n = short(r["Kernel_Name"])
    gy = int(r.get("Grid_Size_Y", r.get("Grid_Size", "1")) or 1)
    if n == "k_nn_partial" and "Grid_Size_Y" in r:
        n += " (full sweep)" if gy > 8 else " (delta sweep)"
    return n


def main(dirs):
    tr = glob.glob(os.path.join(dirs[0], "*kernel_trace.csv"))[0]
    rows = list(csv.DictReader(open(tr)))
    agg = defaultdict(list)
    for r in rows:
        agg[key(r)].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    print("| kernel | launches | mean us | min us | max us | last-20 mean us |")
    print("|---|---|---|---|---|---|")
    for k, v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
        last = v[-20:]
        print("| %s | %d | %.1f | %.1f | %.1f | %.1f |" % (k, len(v), sum(v) / len(v), min(v), max(v),
                                                        sum(last) / len(last)))
    for d in dirs[1:]:
        f = glob.glob(os.path.join(d, "*counter_collection.csv"))[0]
        pm = list(csv.DictReader(open(f)))
        per = defaultdict(list)
        for r in pm:
            n = short(r["Kernel_Name"])
            if n == "k_nn_partial":
                n += " (full sweep)" if int(r["Grid_Size"]) > 2048 * 8 else " (delta sweep)"
            per[(n, r["Counter_Name"])].append(float(r["Counter_Value"]))
        print()
        print("| kernel | counter | launches | last-20 mean per launch |")
        print("|---|---|---|---|")
        for (n, c), v in sorted(per.items()):
            last = v[-20:]
            print("| %s | %s | %d | %.1f |" % (n, c, len(v), sum(last) / len(last)))


if __name__ == "__main__":
    main(sys.argv[1:])
