# Needs a lab build (scripts/build_variants.sh / build_variant_src.sh with -DTPL_LAB=1): the
# product library ignores the TPL_SLICES layout knob.
set -u
cd ${GRAFT_REPO_ROOT:-$(pwd)}
V=$PWD/two-pass-lanczos_amd/variants/libtpl_s16.so
run() { out=$(env "$@" timeout -k 10 300 python bench.py --other-configs 0 --one-pass 0 --pcie 0 --scale-ref 0 --cpu-baseline 0 --steps 10 2>/dev/null | tail -1); python3 -c "import json,sys; d=json.loads(sys.argv[1]); r=d['roofline']; print(sys.argv[2], d['ms_per_solve_median'], r['pass1_us_per_step'], r['avg_launch_us_events'], r['kernels_us_isolated'], d['config']['x_sha256_16'])" "$out" "$*"; }
for rep in 1 2; do
  run X=base
  run TPL_LIB_PATH=$V
  run TPL_LIB_PATH=$V TPL_SLICES=16
done
