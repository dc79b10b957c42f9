#!/bin/bash
# Round record of the default bench: the driver's command (PMC passes + CPU baseline) and a
# rocprofv3 --kernel-trace --stats summary of the same command.  Outputs gpurun_out/rec_$1/.
T=$1
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/rec_$T; mkdir -p $O
timeout -k 10 400 python $R/bench.py > $O/bench.json 2> $O/bench.err &&
cd /tmp && export TMPDIR=/tmp &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $R/bench.py --no-pmc --no-cpu > $O/prof_bench.json 2> $O/prof_bench.err
