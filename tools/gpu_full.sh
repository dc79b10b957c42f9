# Round record on one MI355X: parity tests, cfg2 bench (+ rocprofv3 kernel trace, HBM PMC passes),
# cfg3 bench, cfg4 LOS batch.  Outputs under gpurun_out/full/.
set -o pipefail
R="$GRAFT_REPO_ROOT"; O="$R/gpurun_out/full"
export TMPDIR=/tmp
mkdir -p "$O" && cd "$R"
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread > "$O/pytest_gpu.log" 2>&1 && echo "pytest ok" &&
timeout -k 10 300 python bench.py > "$O/bench_cfg2.json" 2> "$O/bench_cfg2.err" && echo "cfg2 ok" &&
timeout -k 10 300 python tools/bench_los.py 10000 200 > "$O/bench_cfg4.json" 2> "$O/bench_cfg4.err" && echo "cfg4 ok" &&
timeout -k 10 400 python bench.py --config cfg3 --steps 5 --warmup 1 --no-cpu > "$O/bench_cfg3.json" 2> "$O/bench_cfg3.err" && echo "cfg3 ok" &&
cd /tmp &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof" -o run -- python3 "$R/bench.py" --no-cpu --no-pmc > "$O/prof_bench.json" 2> "$O/prof_bench.err" &&
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$O/pmc_f" -o run -- python3 "$R/bench.py" --no-cpu --no-pmc > "$O/pmc_f.log" 2>&1 &&
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$O/pmc_w" -o run -- python3 "$R/bench.py" --no-cpu --no-pmc > "$O/pmc_w.log" 2>&1 &&
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_los" -o run -- python3 "$R/tools/bench_los.py" 10000 200 > "$O/prof_los.json" 2>&1 &&
echo done
