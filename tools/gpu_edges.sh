# Edge-case parity tests, then the multi-rank rehearsals of the bench on one GPU: the engine's RCCL
# communicator at N=1 (--force-comm) and two ranks on GPU 0 over gloo (--same-device).
set -o pipefail
R="$GRAFT_REPO_ROOT"; O="$R/gpurun_out/edges"
export TMPDIR=/tmp
mkdir -p "$O" && cd "$R"
timeout -k 10 300 python -u -m pytest tests/test_gpu_edges.py -m gpu -x -v --timeout 120 --timeout-method thread > "$O/pytest_edges.log" 2>&1 && echo "edges ok" &&
timeout -k 10 200 python bench.py --force-comm --no-cpu --steps 10 > "$O/bench_forcecomm.json" 2> "$O/bench_forcecomm.err" && echo "force-comm ok" &&
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --same-device --backend gloo --no-cpu --steps 10 > "$O/bench_w2_gloo.json" 2> "$O/bench_w2_gloo.err" && echo "w2 ok" &&
echo done
