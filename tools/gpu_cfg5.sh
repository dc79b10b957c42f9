set -o pipefail
R="$GRAFT_REPO_ROOT"; O="$R/gpurun_out/cfg5"
export TMPDIR=/tmp
mkdir -p "$O" && cd "$R"
timeout -k 10 500 python -u -m pytest tests/test_gpu_bench_parity.py -m gpu -x -v --timeout 400 --timeout-method thread --durations=8 -k "sharded or book" > "$O/pytest_cfg5.log" 2>&1 ; rc=$?
tail -25 "$O/pytest_cfg5.log"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu --no-pmc --no-events --batch 32768 --steps 20 > "$O/b32k.json" 2> "$O/b32k.err" && python3 -c "
import json; d=json.load(open('$O/b32k.json')); print('b32k', d['value'], d['ms_per_step'], d['host_us_per_step'])"
