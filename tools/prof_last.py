"""Durations of the last N dispatches of each kernel in a rocprofv3 --kernel-trace run:
python tools/prof_last.py DIR [N]."""
import csv
import glob
import os
import sys

d = sys.argv[1]
n = int(sys.argv[2]) if len(sys.argv) > 2 else 5
rows = list(csv.DictReader(open(glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)[0])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
by = {}
for r in rows:
    by.setdefault(r["Kernel_Name"].split("(")[0], []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for k, v in sorted(by.items(), key=lambda kv: -sum(kv[1][-n:])):
    print("  %-28s last %d: %s us" % (k[:28], n, " ".join("%.0f" % x for x in v[-n:])))
