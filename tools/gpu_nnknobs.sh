# k_nn_pass1 at cfg2 size (N = 75k, B = 4096) over the sweep's chunking knobs.
set -o pipefail
R="$GRAFT_REPO_ROOT"; O="$R/gpurun_out/nnknobs"
export TMPDIR=/tmp
mkdir -p "$O" && cd /tmp
for U in 128 256 512 1024; do for G in 256 512 1024; do
  TR_NN_UNITS=$U TR_NN_GRID=$G timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/u${U}_g${G}" -o run -- python3 "$R/tools/nn_iso.py" 75000 4096 10 > "$O/u${U}_g${G}.log" 2>&1 || exit 1
done; done
for M in 256 512; do
  TR_NN_MAXCHUNK=$M TR_NN_UNITS=2048 TR_NN_GRID=1024 timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/m${M}" -o run -- python3 "$R/tools/nn_iso.py" 75000 4096 10 > "$O/m${M}.log" 2>&1 || exit 1
done
echo done
