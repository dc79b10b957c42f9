# One GPU session: parity tests, isolated NN timing, cfg2 bench, rocprofv3 kernel trace and the
# HBM PMC passes of the same bench (FETCH_SIZE / WRITE_SIZE in separate runs).  Outputs: gpurun_out/.
set -o pipefail
R="$GRAFT_REPO_ROOT"; O="$R/gpurun_out"
export TMPDIR=/tmp
mkdir -p "$O" && cd "$R"
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread > "$O/pytest_gpu.log" 2>&1 && echo "pytest ok" &&
cd /tmp &&
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/nniso_mfma" -o run -- python3 "$R/tools/nn_iso.py" 75000 4096 30 > "$O/nniso_mfma_prof.log" 2>&1 &&
TR_NN_VALU=1 timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/nniso_valu" -o run -- python3 "$R/tools/nn_iso.py" 75000 4096 30 > "$O/nniso_valu_prof.log" 2>&1 &&
cd "$R" && timeout -k 10 300 python bench.py > "$O/bench.json" 2> "$O/bench.err" && echo "bench ok" &&
cd /tmp &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof" -o run -- python3 "$R/bench.py" --no-cpu > "$O/prof_bench.json" 2> "$O/prof_bench.err" &&
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$O/pmc_f" -o run -- python3 "$R/bench.py" --no-cpu > "$O/pmc_f.log" 2>&1 &&
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$O/pmc_w" -o run -- python3 "$R/bench.py" --no-cpu > "$O/pmc_w.log" 2>&1 &&
echo done
