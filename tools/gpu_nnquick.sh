# Quick NN check: parity tests of the sweep, isolated timings at three sizes, the cfg2 bench.
set -o pipefail
R="$GRAFT_REPO_ROOT"; O="$R/gpurun_out/nnquick"
export TMPDIR=/tmp
mkdir -p "$O" && cd "$R"
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -k "nn or cfg3" --timeout 180 --timeout-method thread > "$O/pytest.log" 2>&1 && echo "pytest ok" &&
cd /tmp && for BN in "4096 75000" "4096 1000000" "65536 1000000"; do set -- $BN
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/b$1_n$2" -o run -- python3 "$R/tools/nn_iso.py" $2 $1 10 > "$O/b$1_n$2.log" 2>&1 || exit 1
done && cd "$R" && timeout -k 10 300 python bench.py --no-cpu > "$O/bench.json" 2> "$O/bench.err" && echo done
