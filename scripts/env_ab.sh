#!/bin/bash
# A/B of environment settings on one box: the quick headline bench (no side legs) under
# each "NAME=VALUE" (or "base"), alternated REPS times. Prints median ms, pass one per
# step, live k_p2_spmv, the isolated kernels and x's digest.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
for rep in $(seq 1 ${REPS:-2}); do
  for v in "$@"; do
    if [ "$v" = base ]; then e=""; else e="$v"; fi
    out=$(env $e timeout -k 10 300 python bench.py --other-configs 0 --one-pass 0 --pcie 0 --scale-ref 0 --cpu-baseline 0 --steps 10 2>/dev/null | tail -1)
    python3 -c "import json,sys; d=json.loads(sys.argv[1]); r=d.get('roofline_live', d['roofline']); print('$v', d['ms_per_solve_median'], r['pass1_us_per_step'], r['avg_launch_us_events'], r['kernels_us_isolated'], d['config']['x_sha256_16'])" "$out"
  done
done
