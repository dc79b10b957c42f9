# NN sweep scaling: k_nn_pass1 (MFMA) and k_nn_pass1_valu over tree sizes and batch sizes.
set -o pipefail
R="$GRAFT_REPO_ROOT"; O="$R/gpurun_out/nnsweep"
export TMPDIR=/tmp
mkdir -p "$O" && cd /tmp
for B in 4096 65536; do for N in 20000 75000 300000 1000000; do for V in 0 1; do
  TR_NN_VALU=$V timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/b${B}_n${N}_v${V}" -o run -- python3 "$R/tools/nn_iso.py" $N $B 10 > "$O/b${B}_n${N}_v${V}.log" 2>&1 || exit 1
done; done; done
echo done
