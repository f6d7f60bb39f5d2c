#!/bin/bash
# A/B of the pinned locality-order group count on the headline (bench.py --order-groups G),
# alternated REPS times; prints median ms, pass one us/step, live k_p2_spmv, x digest.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
for rep in $(seq 1 ${REPS:-3}); do
  for g in "$@"; do
    out=$(timeout -k 10 300 python bench.py --order-groups $g --other-configs 0 --one-pass 0 --pcie 0 --scale-ref 0 --cpu-baseline 0 --steps 10 2>/dev/null | tail -1)
    python3 -c "import json,sys; d=json.loads(sys.argv[1]); r=d['roofline']; print('$g', d['ms_per_solve_median'], r['pass1_us_per_step'], r['avg_launch_us_events'], r['kernels']['k_p2_spmv']['avg_launch_us_events'], d['config']['x_sha256_16'])" "$out"
  done
done
