"""Per-kernel mean durations (last N batches) from a rocprofv3 --kernel-trace CSV directory."""
import csv
import glob
import sys
from collections import defaultdict

d = sys.argv[1]
last = int(sys.argv[2]) if len(sys.argv) > 2 else 10
rows = list(csv.DictReader(open(glob.glob(d + "/*kernel_trace.csv")[0])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if "k_samples" in r["Kernel_Name"]]
sub = rows[idx[-last]:] if len(idx) >= last else rows
agg = defaultdict(list)
for r in sub:
    agg[r["Kernel_Name"].split("(")[0].replace("tr::", "")].append(
        (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
span = (int(sub[-1]["End_Timestamp"]) - int(sub[0]["Start_Timestamp"])) / 1e3 / last
tot = 0
for k, v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
    tot += sum(v) / last
    print("%-30s n=%3d mean=%7.1f us" % (k, len(v), sum(v) / len(v)))
print("kernel sum per batch %.1f us, wall span per batch %.1f us" % (tot, span))
