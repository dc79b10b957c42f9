#!/bin/bash
# Per-rank costs that grow with the world size, measured on one GPU: cfg2 without look-ahead
# (stage 0: no correction, the NN on the batch's own stream), and the global-batch kernels of a
# W = 8 step (k_dd over 32768 records, k_expand_arc's correction over the nodes of a 32768-sample
# batch) from a --batch 32768 run under rocprofv3.  Outputs gpurun_out/scale_$1/.
T=$1; R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/scale_$T; mkdir -p $O
timeout -k 10 200 python $R/bench.py --no-pmc --no-cpu --stage 0 > $O/stage0.json 2> $O/stage0.err &&
timeout -k 10 200 python $R/bench.py --no-pmc --no-cpu --stage 1 > $O/stage1.json 2> $O/stage1.err &&
cd /tmp && export TMPDIR=/tmp &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/b32k -o run -- python3 $R/bench.py --no-pmc --no-cpu --batch 32768 --steps 20 > $O/b32k.json 2> $O/b32k.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/b32k_s0 -o run -- python3 $R/bench.py --no-pmc --no-cpu --batch 32768 --steps 20 --stage 0 > $O/b32k_s0.json 2> $O/b32k_s0.err
