# SQ / GRBM counters of k_nn_pass1 (MFMA) on the isolated cfg2-size sweep, one --pmc pass each.
set -o pipefail
R="$GRAFT_REPO_ROOT"; O="$R/gpurun_out/nnpmc"
export TMPDIR=/tmp
mkdir -p "$O" && cd /tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU --output-format csv -d "$O/sq" -o run -- python3 "$R/tools/nn_iso.py" 75000 4096 10 > "$O/sq.log" 2>&1 &&
timeout -s KILL 90 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d "$O/grbm" -o run -- python3 "$R/tools/nn_iso.py" 75000 4096 10 > "$O/grbm.log" 2>&1 &&
timeout -s KILL 90 rocprofv3 --pmc SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_MFMA SQ_INSTS_SALU --output-format csv -d "$O/sq2" -o run -- python3 "$R/tools/nn_iso.py" 75000 4096 10 > "$O/sq2.log" 2>&1
echo rc=$?
