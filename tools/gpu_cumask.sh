# CU-masked main chain (TR_MAIN_CUS) A/B on the cfg2 bench, after the pipelined parity tests under
# the mask.  Outputs under gpurun_out/cumask/.
set -o pipefail
R="$GRAFT_REPO_ROOT"; O="$R/gpurun_out/cumask"
export TMPDIR=/tmp
mkdir -p "$O" && cd "$R"
TR_MAIN_CUS=128 timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -k "pipelined or cfg3_batches or rrt_api or batched_rrt" --timeout 180 --timeout-method thread > "$O/pytest.log" 2>&1 || { echo "pytest FAIL"; tail -5 "$O/pytest.log"; exit 1; }
echo "pytest $(tail -1 "$O/pytest.log")"
run() {  # name, env... (then bench args after --)
  local n=$1; shift
  env "$@" timeout -k 10 120 python bench.py --no-cpu > "$O/$n.json" 2> "$O/$n.err" || exit 1
  echo "$n $(python -c "import json; d=json.loads(open('$O/$n.json').read().splitlines()[-1]); print(round(d['value']/1e6,2), round(d['ms_per_step']*1e3,1), round(d['roofline']['frac'],3))")"
}
for k in 1 2; do
  run off.$k X=0
  run m192.$k TR_MAIN_CUS=192
  run m128.$k TR_MAIN_CUS=128
  run m96.$k TR_MAIN_CUS=96
  run m64.$k TR_MAIN_CUS=64
done
(cd /tmp && TR_MAIN_CUS=128 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_m128" -o run -- python3 "$R/bench.py" --no-cpu > "$O/prof_m128.json" 2> "$O/prof_m128.err") && python tools/ktimes.py "$O/prof_m128" 20 &&
echo done
