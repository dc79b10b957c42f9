# GPU parity tests, then cfg2 and cfg3 benches with their PMC traffic passes.
set -o pipefail
R="$GRAFT_REPO_ROOT"; O="$R/gpurun_out/${1:-r3c}"
export TMPDIR=/tmp
mkdir -p "$O" && cd "$R"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread > "$O/pytest_gpu.log" 2>&1 ; rc=$?
tail -4 "$O/pytest_gpu.log"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu > "$O/bench_cfg2.json" 2> "$O/bench_cfg2.err" && echo "cfg2 ok" && cut -c1-330 "$O/bench_cfg2.json" &&
timeout -k 10 400 python bench.py --config cfg3 --steps 5 --warmup 1 --no-cpu > "$O/bench_cfg3.json" 2> "$O/bench_cfg3.err" && echo "cfg3 ok" && cut -c1-330 "$O/bench_cfg3.json"
