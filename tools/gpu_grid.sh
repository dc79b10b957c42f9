# k_nn_pass1 grid cap (TR_NN_GRID) under the depth-2 pipeline: the sweep's blocks hold every VGPR
# of their SIMDs (256 VGPRs x 2 waves), so the cap decides how much of the chip the batch's own
# kernels can use meanwhile.  Outputs under gpurun_out/grid/.
set -o pipefail
R="$GRAFT_REPO_ROOT"; O="$R/gpurun_out/grid"
export TMPDIR=/tmp
mkdir -p "$O" && cd "$R"
run() {  # name, env...
  local n=$1; shift
  env "$@" timeout -k 10 120 python bench.py --no-cpu --steps 20 > "$O/$n.json" 2> "$O/$n.err" || exit 1
  echo "$n $(python -c "import json,sys; d=json.loads(open('$O/$n.json').read().splitlines()[-1]); print(round(d['value']/1e6,2), round(d['ms_per_step']*1e3,1), round(d['roofline']['frac'],3), round(d['roofline']['launch_us'],1))")"
}
for G in 512 384 256 192 128 96 64; do run g$G TR_NN_GRID=$G; done
for G in 512 256 128; do run g${G}_u1024 TR_NN_GRID=$G TR_NN_UNITS=1024; done
run g512b TR_NN_GRID=512
echo done
