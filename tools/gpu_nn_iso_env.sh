#!/bin/bash
# Isolated NN kernels (tools/nn_iso.py, cfg2 size) under rocprofv3 for environment variants:
# bash tools/gpu_nn_iso_env.sh TAG "ENV..." ... ("-" = none).  gpurun_out/nnenv_TAG/v<i>/.
T=$1; shift
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/nnenv_$T; mkdir -p $O; cd /tmp && export TMPDIR=/tmp
i=0
for v in "$@"; do
  e=""; [ "$v" != "-" ] && e="$v"
  env $e timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/v$i -o run -- python3 $R/tools/nn_iso.py 75000 4096 40 > $O/v$i.log 2>&1 || exit 1
  i=$((i+1))
done
