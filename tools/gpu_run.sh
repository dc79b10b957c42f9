set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 && echo "pytest ok" &&
timeout -k 10 120 python tools/nn_iso.py 75000 4096 30 > gpurun_out/nniso_mfma.log 2>&1 &&
cd /tmp && timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/nniso_mfma -o run -- python3 $GRAFT_REPO_ROOT/tools/nn_iso.py 75000 4096 30 > $GRAFT_REPO_ROOT/gpurun_out/nniso_mfma_prof.log 2>&1 &&
TR_NN_VALU=1 timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/nniso_valu -o run -- python3 $GRAFT_REPO_ROOT/tools/nn_iso.py 75000 4096 30 > $GRAFT_REPO_ROOT/gpurun_out/nniso_valu_prof.log 2>&1 &&
cd $GRAFT_REPO_ROOT && timeout -k 10 300 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err &&
timeout -k 10 300 python bench.py --stage 2 --no-cpu > gpurun_out/bench_s2.json 2> gpurun_out/bench_s2.err &&
echo done
