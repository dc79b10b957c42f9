# cfg2 bench under rocprofv3 --kernel-trace --stats (the kernel summary goes to profiles/)
set -o pipefail
R="$GRAFT_REPO_ROOT"; O="$R/gpurun_out/${1:-prof}"
export TMPDIR=/tmp
mkdir -p "$O" && cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof" -o run -- python3 "$R/bench.py" --no-cpu --no-pmc > "$O/prof_bench.json" 2> "$O/prof_bench.err" ; rc=$?
cut -c80-130 "$O/prof_bench.json"
python3 - <<P
import csv,glob
f=glob.glob("$O/prof/**/*kernel_stats.csv",recursive=True)
for r in list(csv.DictReader(open(f[0])))[:16]:
    print("%-34s calls %5s avg %8.1f min %8.1f max %8.1f us %6s%%" % (r["Name"].split("(")[0][:34], r["Calls"], float(r["AverageNs"])/1e3, float(r["MinNs"])/1e3, float(r["MaxNs"])/1e3, r["Percentage"]))
P
rm -f "$O"/prof/*kernel_trace.csv
exit $rc
