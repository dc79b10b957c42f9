# cfg2 bench under side-stream sweep grid caps, and the Theta* timing with pinned staging.
set -o pipefail
R="$GRAFT_REPO_ROOT"; O="$R/gpurun_out/knobs"
export TMPDIR=/tmp
mkdir -p "$O" && cd "$R"
timeout -k 10 200 python tools/bench_astar.py > "$O/bench_astar.json" 2> "$O/bench_astar.err" || exit 1
for G in 128 256 384 512 1024; do
  TR_NN_GRID=$G timeout -k 10 200 python bench.py --no-cpu > "$O/bench_g$G.json" 2> "$O/bench_g$G.err" || exit 1
done
TR_NN_VALU=1 timeout -k 10 200 python bench.py --no-cpu > "$O/bench_valu.json" 2> "$O/bench_valu.err" || exit 1
echo done
