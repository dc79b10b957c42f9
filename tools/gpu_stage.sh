# Look-ahead depth / commit lag A/B on the cfg2 bench.  Outputs under gpurun_out/stage/.
set -o pipefail
R="$GRAFT_REPO_ROOT"; O="$R/gpurun_out/stage"
export TMPDIR=/tmp
mkdir -p "$O" && cd "$R"
run() {  # name, bench args...
  local n=$1; shift
  timeout -k 10 120 python bench.py --no-cpu --steps 40 "$@" > "$O/$n.json" 2> "$O/$n.err" || exit 1
  echo "$n $(python -c "import json,sys; d=json.loads(open('$O/$n.json').read().splitlines()[-1]); print(round(d['value']/1e6,2), round(d['ms_per_step']*1e3,1), round(d['roofline']['frac'],3))")"
}
run s1 --stage 1
run s2 --stage 2
run s0 --stage 0
run s2_lag5 --stage 2 --lag 5
run s2_lag3 --stage 2 --lag 3
run s1_lag5 --stage 1 --lag 5
run s2b --stage 2
TR_TRACE=1 timeout -k 10 120 python bench.py --no-cpu --steps 40 --stage 2 > "$O/s2trace.json" 2> "$O/s2trace.err" &&
echo done
