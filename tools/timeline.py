"""Print the kernel timeline (start/end us relative to the first shown kernel) of the last launches
in a rocprofv3 --kernel-trace CSV directory: python tools/timeline.py DIR [N]."""
import csv
import glob
import sys

d = sys.argv[1]
last = int(sys.argv[2]) if len(sys.argv) > 2 else 40
rows = list(csv.DictReader(open(glob.glob(d + "/*kernel_trace.csv")[0])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
rows = rows[-last:]
t0 = int(rows[0]["Start_Timestamp"])
for r in rows:
    s, e = int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0
    name = r["Kernel_Name"].split("(")[0].replace("tr::", "").replace("void ", "")
    print("%9.1f %9.1f %7.1f  q%-3s %s" % (s / 1e3, e / 1e3, (e - s) / 1e3, r.get("Queue_Id", r.get("Stream_Id", "?")), name))
