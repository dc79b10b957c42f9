#!/bin/bash
# A/B of environment knobs on the default bench: bash tools/gpu_ab_env.sh TAG "ENV1" "ENV2" ...
# ("-" = no extra env).  Each variant runs bench.py --no-pmc --no-cpu twice, interleaved.
# Outputs gpurun_out/ab_TAG/<i>_<rep>.json (+ .err).
T=$1; shift
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/ab_$T; mkdir -p $O
for rep in 0 1; do
  i=0
  for v in "$@"; do
    e=""; [ "$v" != "-" ] && e="$v"
    echo "variant $i ($v) rep $rep"
    env $e timeout -k 10 200 python $R/bench.py --no-pmc --no-cpu > $O/${i}_$rep.json 2> $O/${i}_$rep.err || exit $?
    i=$((i+1))
  done
done
