#!/bin/bash
# k_nn_pass1 software-pipelined MFMA stream A/B: isolated NN (default / swp / swp+sched hints),
# the GPU NN parity tests with the swp+hints build, and the default bench with it.
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/nnswp; mkdir -p $O; cd $R
bash tools/gpu_nn_iso_ab.sh swp - theta-rrt_amd/variants/libthetarrt_swp.so theta-rrt_amd/variants/libthetarrt_swpsgb.so &&
cd $R && THETARRT_LIB=$R/theta-rrt_amd/variants/libthetarrt_swpsgb.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_edges.py -x -q --timeout 180 --timeout-method thread -k "nn or cfg2 or cfg3" > $O/pytest.log 2>&1 && echo pytest ok &&
THETARRT_LIB=$R/theta-rrt_amd/variants/libthetarrt_swpsgb.so timeout -k 10 300 python bench.py --no-pmc --no-cpu > $O/bench_swpsgb.json 2> $O/bench_swpsgb.err &&
timeout -k 10 300 python bench.py --no-pmc --no-cpu > $O/bench_default.json 2> $O/bench_default.err && echo done
