set -u
for rep in $(seq 1 ${REPS:-4}); do
  for v in base "$@"; do
    if [ $v = base ]; then lib=""; else lib="TPL_LIB_PATH=$PWD/two-pass-lanczos_amd/variants/libtpl_$v.so"; fi
    out=$(env $lib timeout -k 10 300 python bench.py --arcs 5000000 --headline-only 1 --steps 3 2>/dev/null | tail -1)
    python3 -c "import json,sys; d=json.loads(sys.argv[1]); r=d['roofline']; print('$v', d['ms_per_solve_median'], r['pass1_us_per_step'], r['avg_launch_us_events'], d['config']['x_sha256_16'])" "$out"
  done
done
