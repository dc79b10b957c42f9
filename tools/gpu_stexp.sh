# Look-ahead scope A/B under depth 1/2: nearest nodes only (default) vs the whole expansion on the
# side stream (TR_STAGE_EXPAND=1, re-expanding only changed samples), plus the pipelined parity
# tests under TR_STAGE_EXPAND=1.  Outputs under gpurun_out/stexp/.
set -o pipefail
R="$GRAFT_REPO_ROOT"; O="$R/gpurun_out/stexp"
export TMPDIR=/tmp
mkdir -p "$O" && cd "$R"
run() {  # name, steps, env... -- args
  local n=$1; local k=$2; shift 2
  env "$@" timeout -k 10 120 python bench.py --no-cpu --steps $k > "$O/$n.json" 2> "$O/$n.err" || exit 1
  echo "$n $(python -c "import json,sys; d=json.loads(open('$O/$n.json').read().splitlines()[-1]); print(round(d['value']/1e6,2), round(d['ms_per_step']*1e3,1), round(d['roofline']['frac'],3))")"
}
run nn_s2 20 X=1
run ex_s2 20 TR_STAGE_EXPAND=1
run nn_s2b 20 X=2
run ex_s2b 20 TR_STAGE_EXPAND=1
run ex_s2_40 40 TR_STAGE_EXPAND=1
run nn_s2_40 40 X=1
TR_STAGE_EXPAND=1 timeout -k 10 300 python -u -m pytest tests -m gpu -x -v -k "pipelined or sharded or cfg3_batches or cfg5" --timeout 180 --timeout-method thread > "$O/pytest_stexp.log" 2>&1 && echo "pytest stexp ok" &&
cd /tmp && TR_STAGE_EXPAND=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof" -o run -- python3 "$R/bench.py" --no-cpu > "$O/prof_bench.json" 2> "$O/prof_bench.err" &&
echo done
