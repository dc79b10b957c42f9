set -o pipefail
R="$GRAFT_REPO_ROOT"; O="$R/gpurun_out/rng"
export TMPDIR=/tmp
mkdir -p "$O" && cd "$R"
timeout -k 10 400 python -u -m pytest tests/test_rng.py -m gpu -x -v --timeout 180 --timeout-method thread > "$O/pytest_rng.log" 2>&1 ; rc=$?
tail -12 "$O/pytest_rng.log"
[ $rc -eq 0 ] || exit $rc
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof32k" -o run -- python3 "$R/bench.py" --no-cpu --no-pmc --no-events --batch 32768 --steps 20 > "$O/b32k.json" 2> "$O/b32k.err" ; rc=$?
cut -c1-300 "$O/b32k.json"; tail -2 "$O/b32k.err"
python3 - <<P
import csv,glob
f=glob.glob("$O/prof32k/**/*kernel_stats.csv",recursive=True)
for r in list(csv.DictReader(open(f[0])))[:14]:
    print("%-40s calls %5s avg %10.1f us  %5s%%" % (r["Name"].split("(")[0][:40], r["Calls"], float(r["AverageNs"])/1e3, r["Percentage"]))
P
exit $rc
