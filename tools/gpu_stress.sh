#!/bin/bash
# Repeated default-bench runs of a library build (stress for rare pipeline errors):
# bash tools/gpu_stress.sh TAG N [ENV...]; stops at the first failing run.  gpurun_out/stress_TAG/.
T=$1; N=$2; shift 2
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/stress_$T; mkdir -p $O
for i in $(seq 1 $N); do
  env "$@" timeout -k 10 200 python $R/bench.py --no-pmc --no-cpu > $O/$i.json 2> $O/$i.err || { echo "run $i failed"; exit 1; }
  echo "run $i ok"
done
