# Diagnosis build TR_DIAG_RESOLVE (not a parity build): chunks rescanned per sample by
# k_nn_resolve in the cfg2 bench vs the isolated uniform tree.  Outputs under gpurun_out/diagres/.
set -o pipefail
R="$GRAFT_REPO_ROOT"; O="$R/gpurun_out/diagres"
export TMPDIR=/tmp
mkdir -p "$O" && cd "$R"
cp theta-rrt_amd/libthetarrt.so "$O/orig.so.keep"
cp theta-rrt_amd/variants/libthetarrt_diagres.so theta-rrt_amd/libthetarrt.so &&
timeout -k 10 120 python bench.py --no-cpu > "$O/bench.json" 2> "$O/bench.err"
rc=$?
timeout -k 10 120 python tools/nn_iso.py 75000 4096 3 > "$O/iso.log" 2>&1
cp "$O/orig.so.keep" theta-rrt_amd/libthetarrt.so && rm -f "$O/orig.so.keep"
grep -c TR_DIAG "$O/bench.err" || true
grep TR_DIAG "$O/bench.err" | tail -14 || true
grep TR_DIAG "$O/iso.log" | tail -2 || true
exit $rc
