# Theta*/A* on the engine: parity tests, then the search timing tool.
set -o pipefail
R="$GRAFT_REPO_ROOT"; O="$R/gpurun_out/astar"
export TMPDIR=/tmp
mkdir -p "$O" && cd "$R"
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v -k "astar or search or findnearest" --timeout 180 --timeout-method thread > "$O/pytest.log" 2>&1 && echo "pytest ok" &&
timeout -k 10 300 python tools/bench_astar.py > "$O/bench_astar.json" 2> "$O/bench_astar.err" && echo done
