#!/bin/bash
# k_nn_pass1 block shape A/B: 4 waves x 16 sample tiles (default) vs 8 waves x 8 tiles (4 waves per
# SIMD): isolated NN, the NN GPU tests with the variant, the default bench with each build.
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/nnmt; mkdir -p $O; cd $R
V=$R/theta-rrt_amd/variants/libthetarrt_mt8.so
bash tools/gpu_nn_iso_ab.sh mt - theta-rrt_amd/variants/libthetarrt_mt8.so &&
cd $R && THETARRT_LIB=$V timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_edges.py -x -q --timeout 180 --timeout-method thread -k "nn or cfg2 or cfg3" > $O/pytest.log 2>&1 && echo pytest ok &&
THETARRT_LIB=$V timeout -k 10 300 python bench.py --no-pmc --no-cpu > $O/bench_mt8.json 2> $O/bench_mt8.err &&
timeout -k 10 300 python bench.py --no-pmc --no-cpu > $O/bench_default.json 2> $O/bench_default.err && echo done
