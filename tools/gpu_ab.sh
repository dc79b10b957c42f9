# A/B of engine options on the cfg2 bench: gpu_ab.sh <name> "<args A>" "<args B>" ... (each run
# without the CPU baseline; PMC traffic passes included unless the args say --no-pmc)
set -o pipefail
R="$GRAFT_REPO_ROOT"; O="$R/gpurun_out/$1"; shift
export TMPDIR=/tmp
mkdir -p "$O" && cd "$R"
i=0
for a in "$@"; do
  timeout -k 10 300 python bench.py --no-cpu $a > "$O/run$i.json" 2> "$O/run$i.err" || exit $?
  python3 - "$O/run$i.json" "$a" <<'P'
import json, sys
d = json.load(open(sys.argv[1]))
r = d.get("roofline", {})
print("[%s] value %.2fM median %.2fM us/step %.1f kernels %s traffic %s" % (
    sys.argv[2], d["value"] / 1e6, d["window_rates"]["median"] / 1e6, d["ms_per_step"] * 1e3,
    {k: round(v, 1) for k, v in d.get("kernel_us", {}).items()}, r.get("traffic")))
P
  i=$((i+1))
done
