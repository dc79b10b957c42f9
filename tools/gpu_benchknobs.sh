# cfg2 bench under the pipeline's knobs (one JSON line each) and one TR_TRACE run (host timestamps
# per batch on stderr).  Outputs under gpurun_out/bknobs/.
set -o pipefail
R="$GRAFT_REPO_ROOT"; O="$R/gpurun_out/bknobs"
export TMPDIR=/tmp
mkdir -p "$O" && cd "$R"
run() {  # name, env..., -- bench args
  local n=$1; shift
  env "$@" timeout -k 10 120 python bench.py --no-cpu --steps 40 > "$O/$n.json" 2> "$O/$n.err" || exit 1
  echo "$n $(python -c "import json,sys; d=json.loads(open('$O/$n.json').read().splitlines()[-1]); print(round(d['value']/1e6,2), round(d['ms_per_step']*1e3,1), round(d['roofline']['frac'],3))")"
}
run base X=1
run trace TR_TRACE=1
run u1024_g512 TR_NN_UNITS=1024
run u1024_g1024 TR_NN_UNITS=1024 TR_NN_GRID=1024
run u256_g256 TR_NN_UNITS=256 TR_NN_GRID=256
run prio_hi TR_SIDE_PRIO=hi
run prio_mid TR_SIDE_PRIO=mid
run base2 X=2
echo done
