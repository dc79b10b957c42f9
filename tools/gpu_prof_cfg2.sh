#!/bin/bash
# cfg2 kernel trace (rocprofv3 --kernel-trace --stats, 40 timed steps) + the bench line of the same
# command.  usage: bash tools/gpu_prof_cfg2.sh TAG [extra bench args]; outputs gpurun_out/prof_TAG/.
T=$1; shift
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/prof_$T; mkdir -p $O; cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o run -- python3 $R/bench.py --no-pmc --no-cpu --steps 40 "$@" > $O/bench.json 2> $O/bench.err
