set -o pipefail
R="$GRAFT_REPO_ROOT"; O="$R/gpurun_out/r3a"
export TMPDIR=/tmp
mkdir -p "$O" && cd "$R"
timeout -k 10 200 python -u -m pytest tests/wip_no_alloc.py -x -v --timeout 120 --timeout-method thread > "$O/pytest_noalloc.log" 2>&1 ; rc=$?
tail -5 "$O/pytest_noalloc.log"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$O/smoke.log" 2>&1 && echo "smoke ok" &&
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > "$O/bench_driver.json" 2> "$O/bench_driver.err" && echo "driver bench ok" && cat "$O/bench_driver.json" | cut -c1-400 &&
timeout -k 10 300 python bench.py --no-cpu --no-pmc > "$O/bench_200.json" 2> "$O/bench_200.err" && echo "bench 200 ok" && cat "$O/bench_200.json" | cut -c1-300 &&
cd /tmp &&
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$O/pmc_f" -o run -- python3 "$R/bench.py" --no-cpu --no-pmc --steps 20 > "$O/pmc_f.log" 2>&1 ; rc=$?
tail -3 "$O/pmc_f.log" | cut -c1-600
echo "pmc rc $rc"
