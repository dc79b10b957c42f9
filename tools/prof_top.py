"""Top kernels of a rocprofv3 --stats run: python tools/prof_top.py DIR [N]."""
import csv
import glob
import json
import os
import sys

d = sys.argv[1]
rows = list(csv.DictReader(open(glob.glob(os.path.join(d, "**", "*kernel_stats.csv"), recursive=True)[0])))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:int(sys.argv[2]) if len(sys.argv) > 2 else 12]:
    print("  %-28s n=%5s avg=%7.1f min=%7.1f max=%7.1f us" % (r["Name"].split("(")[0][:28], r["Calls"],
          float(r["AverageNs"]) / 1e3, float(r["MinNs"]) / 1e3, float(r["MaxNs"]) / 1e3))
b = os.path.join(d, "bench.json")
if os.path.exists(b) and os.path.getsize(b):
    j = json.load(open(b))
    print("  value %.2fM  median %.2fM  ms/step %.3f  host %s" % (j["value"] / 1e6, j["window_rates"]["median"] / 1e6,
          j["ms_per_step"], {k: round(v, 1) for k, v in j["host_us_per_step"].items()}))
