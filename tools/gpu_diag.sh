# Diagnosis builds (NOT parity builds): k_expand_arc with its arc check and/or body rays compiled
# out (TR_DIAG_NOARC / TR_DIAG_NORAYS), kernel trace of the cfg2 bench for each.  Outputs under
# gpurun_out/diag/.  The in-tree library is restored at the end.
set -o pipefail
R="$GRAFT_REPO_ROOT"; O="$R/gpurun_out/diag"
export TMPDIR=/tmp
mkdir -p "$O" && cd "$R"
cp theta-rrt_amd/libthetarrt.so "$O/orig.so.keep"
for V in "$@"; do
  cp "theta-rrt_amd/variants/libthetarrt_$V.so" theta-rrt_amd/libthetarrt.so || exit 1
  (cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_$V" -o run -- python3 "$R/bench.py" --no-cpu > "$O/prof_$V.json" 2> "$O/prof_$V.err") || { echo "$V FAIL"; break; }
  echo "$V $(python tools/ktimes.py "$O/prof_$V" 20 | grep -E 'expand|sum' | tr '\n' ' ')"
done
cp "$O/orig.so.keep" theta-rrt_amd/libthetarrt.so && rm -f "$O/orig.so.keep"
echo done
