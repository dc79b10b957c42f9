# A/B of library builds on the cfg2 bench: gpu_ab_lib.sh <name> <variant|-> ... ("-" = the product
# build); three passes over the list so box drift shows.
set -o pipefail
R="$GRAFT_REPO_ROOT"; O="$R/gpurun_out/$1"; shift
export TMPDIR=/tmp
mkdir -p "$O" && cd "$R"
for pass in 0 1 2; do
for v in "$@"; do
  lib="$R/theta-rrt_amd/libthetarrt.so"; [ "$v" = "-" ] || lib="$R/theta-rrt_amd/libthetarrt_$v.so"
  THETARRT_LIB="$lib" timeout -k 10 300 python bench.py --no-cpu --no-pmc > "$O/$v.$pass.json" 2> "$O/$v.$pass.err" || exit $?
  python3 - "$O/$v.$pass.json" "$v" <<'P'
import json, sys
d = json.load(open(sys.argv[1]))
print("[%s] value %.2fM median %.2fM us/step %.1f kernels %s" % (
    sys.argv[2], d["value"] / 1e6, d["window_rates"]["median"] / 1e6, d["ms_per_step"] * 1e3,
    {k: round(v, 1) for k, v in d.get("kernel_us", {}).items()}))
P
done
done
