"""Per-kernel PMC means over the last N launches from rocprofv3 --pmc CSV directories.

usage: python tools/pmc_table.py N DIR [DIR ...]"""
import csv
import glob
import os
import sys
from collections import defaultdict

last = int(sys.argv[1])
per = defaultdict(list)
for d in sys.argv[2:]:
    f = glob.glob(os.path.join(d, "*counter_collection.csv"))[0]
    for r in csv.DictReader(open(f)):
        n = r["Kernel_Name"].split("(")[0].replace("tr::", "")
        per[(n, r["Counter_Name"])].append(float(r["Counter_Value"]))
names = sorted({k[0] for k in per})
ctrs = sorted({k[1] for k in per})
print("| kernel | " + " | ".join(ctrs) + " |")
print("|---|" + "---|" * len(ctrs))
for n in names:
    vals = []
    for c in ctrs:
        v = per.get((n, c), [])[-last:]
        vals.append("%.4g" % (sum(v) / len(v)) if v else "-")
    print("| %s | %s |" % (n, " | ".join(vals)))
