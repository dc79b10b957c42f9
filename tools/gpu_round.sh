# Full round record on one MI355X: parity tests, smoke(), the driver's bench command and the
# 200-step run, cfg3, cfg4 (LOS batch), Theta* (host search and device-resident batches), the cfg2
# bench under rocprofv3 --kernel-trace --stats and under --pmc (default environment: the engine
# finds the serialized dispatch itself).  Outputs under gpurun_out/<name>/.
set -o pipefail
R="$GRAFT_REPO_ROOT"; O="$R/gpurun_out/${1:-round}"
export TMPDIR=/tmp
mkdir -p "$O" && cd "$R"
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$O/pytest_gpu.log" 2>&1 ; rc=$?
tail -3 "$O/pytest_gpu.log"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$O/smoke.log" 2>&1 && echo "smoke ok" &&
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > "$O/bench_driver.json" 2> "$O/bench_driver.err" && echo "driver bench ok" &&
timeout -k 10 300 python bench.py > "$O/bench_cfg2.json" 2> "$O/bench_cfg2.err" && echo "cfg2 ok" &&
timeout -k 10 300 python tools/bench_los.py 10000 200 > "$O/bench_cfg4.json" 2> "$O/bench_cfg4.err" && echo "cfg4 ok" &&
timeout -k 10 300 python tools/bench_astar.py > "$O/bench_astar.json" 2> "$O/bench_astar.err" && echo "astar ok" &&
timeout -k 10 400 python bench.py --config cfg3 --steps 5 --warmup 1 --no-cpu > "$O/bench_cfg3.json" 2> "$O/bench_cfg3.err" && echo "cfg3 ok" &&
timeout -k 10 300 python bench.py --no-cpu --no-pmc --no-events --batch 32768 --steps 20 > "$O/bench_b32k.json" 2> "$O/bench_b32k.err" && echo "b32k ok" &&
cd /tmp &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof" -o run -- python3 "$R/bench.py" --no-cpu --no-pmc > "$O/prof_bench.json" 2> "$O/prof_bench.err" && rm -f "$O"/prof/*kernel_trace.csv &&
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$O/pmc_f" -o run -- python3 "$R/bench.py" --no-cpu --no-pmc --steps 20 > "$O/pmc_f.log" 2>&1 && rm -rf "$O/pmc_f" &&
echo done
