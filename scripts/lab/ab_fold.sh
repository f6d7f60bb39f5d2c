#!/bin/bash
# A/B on one box: the replicated partition over one RCCL rank with the beta rank total
# folded into k_p1_axpy (base) vs its own launch (two-pass-lanczos_amd/ab/libtpl_nofold.so),
# at configs[4]'s 5M arcs and at the N = 8 per-rank share; alternated REPS times.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
cd "$ROOT"
for rep in $(seq 1 ${REPS:-3}); do
  for v in base nofold; do
    if [ $v = base ]; then lib=""; else lib="TPL_LIB_PATH=$ROOT/two-pass-lanczos_amd/ab/libtpl_$v.so"; fi
    env $lib timeout -k 10 200 python bench.py --gpus 1 --partition 1 --arcs 5000000 --steps 5 --warmup 1 --single-ref 0 --parity 0 > "$OUT/ab_$v.log" 2>&1 || { echo "ab $v failed"; tail -5 "$OUT/ab_$v.log"; exit 2; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print('$v 5M 1-rank', d['ms_per_solve_median'], r['pass1_us_per_step'], r['avg_launch_us_events'], d['config']['x_sha256_16'])" "$OUT/ab_$v.log"
    env $lib timeout -k 10 200 python scripts/rank_share.py --ranks 8 --reps 5 --out "$OUT/ab_share_$v.json" > "$OUT/ab_share_$v.log" 2>&1 || { echo "share $v failed"; tail -5 "$OUT/ab_share_$v.log"; exit 3; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1]))['shares']['8']; o=d['one_rank_replicated']; print('$v N8-share 1-rank', o['ms_per_solve'], o['pass1_us_per_step'], o['pass2_us_per_step'], 'single', d['single_gpu']['ms_per_solve'])" "$OUT/ab_share_$v.json"
  done
done
