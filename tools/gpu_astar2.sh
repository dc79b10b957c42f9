set -o pipefail
R="$GRAFT_REPO_ROOT"; O="$R/gpurun_out/astar"
export TMPDIR=/tmp
mkdir -p "$O" && cd "$R"
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 200 --timeout-method thread -k "astar" > "$O/pytest_astar.log" 2>&1 ; rc=$?
tail -30 "$O/pytest_astar.log"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/bench_astar.py > "$O/bench_astar.json" 2> "$O/bench_astar.err" ; rc=$?
python3 -c "
import json; d=json.load(open('$O/bench_astar.json')); r=d['runs']; print({k:(v['seconds'] if 'seconds' in v else v) for k,v in r.items() if k!='device_resident'}); dv=r['device_resident']; print(dv['single_query_s'], dv['single_query']['expanded'], dv['single_query']['consumed'], dv['single_query']['far_pushes']); print({k:v for k,v in dv.items() if k.startswith('random')})"
exit $rc
