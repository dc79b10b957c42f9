# Pipeline parity tests (edge modes, cfg2 oracle subset, sharded loops) and the cfg2 bench.
set -o pipefail
R="$GRAFT_REPO_ROOT"; O="$R/gpurun_out/${1:-quick}"
export TMPDIR=/tmp
mkdir -p "$O" && cd "$R"
timeout -k 10 600 python -u -m pytest tests/test_gpu_bench_parity.py tests/test_gpu_edges.py -m gpu -x -v --timeout 180 --timeout-method thread > "$O/pytest_gpu.log" 2>&1 ; rc=$?
tail -4 "$O/pytest_gpu.log"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu ${2:-} > "$O/bench_cfg2.json" 2> "$O/bench_cfg2.err" && echo "cfg2 ok" && cut -c1-2600 "$O/bench_cfg2.json"
