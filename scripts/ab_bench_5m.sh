set -u
cd ${GRAFT_REPO_ROOT:-/root/repo}
for rep in 1 2; do
  for v in base plainaxpy; do
    if [ "$v" = base ]; then lib=""; else lib="TPL_LIB_PATH=$PWD/two-pass-lanczos_amd/variants/libtpl_$v.so"; fi
    out=$(env $lib timeout -k 10 300 python bench.py --arcs 5000000 --other-configs 0 --one-pass 0 --pcie 0 --scale-ref 0 --cpu-baseline 0 --steps 3 2>/dev/null | tail -1)
    python3 -c "import json,sys; d=json.loads(sys.argv[1]); r=d.get('roofline_live', d['roofline']); print('$v', d['ms_per_solve_median'], r['pass1_us_per_step'], r['avg_launch_us_events'], r['kernels_us_isolated'], d['config']['x_sha256_16'])" "$out"
  done
done
