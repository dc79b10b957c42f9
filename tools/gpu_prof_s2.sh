# Kernel trace of the cfg2 bench at its default look-ahead depth.  Outputs under gpurun_out/profs2/.
set -o pipefail
R="$GRAFT_REPO_ROOT"; O="$R/gpurun_out/profs2"
export TMPDIR=/tmp
mkdir -p "$O" && cd /tmp &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof" -o run -- python3 "$R/bench.py" --no-cpu > "$O/prof_bench.json" 2> "$O/prof_bench.err" &&
cd "$R" && timeout -k 10 120 python tools/nn_iso.py 75000 4096 30 > "$O/nniso.log" 2>&1 &&
echo done
