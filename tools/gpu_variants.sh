# A/B of build-time variants (theta-rrt_amd/variants/*.so, tools/build_variants.py): each is
# copied over the library, parity-checked on the NN tests, then benched (cfg2, two runs) and its
# isolated k_nn_resolve timed.  Outputs under gpurun_out/variants/.
set -o pipefail
R="$GRAFT_REPO_ROOT"; O="$R/gpurun_out/variants"
export TMPDIR=/tmp
mkdir -p "$O" && cd "$R"
cp theta-rrt_amd/libthetarrt.so "$O/orig.so"
for V in "$@"; do
  cp "theta-rrt_amd/variants/libthetarrt_$V.so" theta-rrt_amd/libthetarrt.so || exit 1
  timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -k "${K_FILTER:-nn or pipelined or cfg3_nn}" --timeout 180 --timeout-method thread > "$O/$V.pytest.log" 2>&1 || { echo "$V pytest FAIL"; exit 1; }
  for k in 1 2; do
    timeout -k 10 120 python bench.py --no-cpu > "$O/$V.$k.json" 2> "$O/$V.$k.err" || exit 1
    echo "$V.$k $(python -c "import json; d=json.loads(open('$O/$V.$k.json').read().splitlines()[-1]); print(round(d['value']/1e6,2), round(d['ms_per_step']*1e3,1), round(d['roofline']['frac'],3))")"
  done
  (cd /tmp && timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/iso_$V" -o run -- python3 "$R/tools/nn_iso.py" 75000 4096 20 > "$O/iso_$V.log" 2>&1) || exit 1
done
cp "$O/orig.so" theta-rrt_amd/libthetarrt.so
echo done
