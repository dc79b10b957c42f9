# Cross-stream event scope (TR_EV_SCOPE) A/B on the cfg2 bench, plus the pipelined parity tests
# under the device-scope edges.  Outputs under gpurun_out/evscope/.
set -o pipefail
R="$GRAFT_REPO_ROOT"; O="$R/gpurun_out/evscope"
export TMPDIR=/tmp
mkdir -p "$O" && cd "$R"
run() {  # name, env...
  local n=$1; shift
  env "$@" timeout -k 10 120 python bench.py --no-cpu --steps 40 > "$O/$n.json" 2> "$O/$n.err" || exit 1
  echo "$n $(python -c "import json,sys; d=json.loads(open('$O/$n.json').read().splitlines()[-1]); print(round(d['value']/1e6,2), round(d['ms_per_step']*1e3,1), round(d['roofline']['frac'],3))")"
}
run sys1 TR_EV_SCOPE=sys
run dev1 TR_EV_SCOPE=dev
run nof1 TR_EV_SCOPE=nofence
run sys2 TR_EV_SCOPE=sys
run dev2 TR_EV_SCOPE=dev
run nof2 TR_EV_SCOPE=nofence
run devtrace TR_EV_SCOPE=dev TR_TRACE=1
TR_EV_SCOPE=dev timeout -k 10 300 python -u -m pytest tests -m gpu -x -v -k "pipelined or sharded or cfg3_batches" --timeout 180 --timeout-method thread > "$O/pytest_dev.log" 2>&1 && echo "pytest dev ok" &&
echo done
