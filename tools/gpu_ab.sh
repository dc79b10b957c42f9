# Full GPU parity suite on the in-tree library, then an interleaved cfg2 bench A/B of two
# build-time variants (theta-rrt_amd/variants/libthetarrt_<A|B>.so), 3 runs each, and the isolated
# expansion kernel of each under the kernel trace.  Outputs under gpurun_out/ab/.
set -o pipefail
R="$GRAFT_REPO_ROOT"; O="$R/gpurun_out/ab"; A=$1; B=$2
export TMPDIR=/tmp
mkdir -p "$O" && cd "$R"
cp theta-rrt_amd/libthetarrt.so "$O/orig.so.keep"
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > "$O/pytest.log" 2>&1 || { echo "pytest FAIL"; tail -5 "$O/pytest.log"; exit 1; }
echo "pytest $(tail -1 "$O/pytest.log")"
for k in 1 2 3; do for V in $A $B; do
  cp "theta-rrt_amd/variants/libthetarrt_$V.so" theta-rrt_amd/libthetarrt.so || exit 1
  timeout -k 10 120 python bench.py --no-cpu > "$O/$V.$k.json" 2> "$O/$V.$k.err" || exit 1
  echo "$V.$k $(python -c "import json; d=json.loads(open('$O/$V.$k.json').read().splitlines()[-1]); print(round(d['value']/1e6,2), round(d['ms_per_step']*1e3,1), round(d['roofline']['frac'],3))")"
done; done
for V in $A $B; do
  cp "theta-rrt_amd/variants/libthetarrt_$V.so" theta-rrt_amd/libthetarrt.so || exit 1
  (cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_$V" -o run -- python3 "$R/bench.py" --no-cpu > "$O/prof_$V.json" 2> "$O/prof_$V.err") || exit 1
done
cp "$O/orig.so.keep" theta-rrt_amd/libthetarrt.so && rm -f "$O/orig.so.keep"
echo done
