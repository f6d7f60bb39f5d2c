#!/bin/bash
# A/B on one box: the headline with the SpMV's two groups of slow bins split at once —
# many-line bins (TPL_SPLIT_LINES) AND many-piece bins (TPL_SPLIT_PIECES), each split in
# two after packing, every other bin in place — in a lab
# build (-DTPL_LAB=1, two-pass-lanczos_amd/ab/libtpl_lab.so) against the product library,
# alternated REPS times. Bin packing never changes a piece's sum: x's digest must not move.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
cd "$ROOT"
LAB=$ROOT/two-pass-lanczos_amd/ab/libtpl_lab.so
for rep in $(seq 1 ${REPS:-3}); do
  for v in base lab0 "s450:100" "s400:64" "s350:48" "s300:32"; do
    case $v in
      base) env_="";;
      lab0) env_="TPL_LIB_PATH=$LAB";;
      s*) w=${v#s}; env_="TPL_LIB_PATH=$LAB TPL_SPLIT_LINES=${w%%:*} TPL_SPLIT_PIECES=${w##*:}";;
    esac
    env $env_ timeout -k 10 120 python bench.py --headline-only 1 --steps 10 --warmup 2 > "$OUT/abc.log" 2>&1 || { echo "run $v failed"; tail -5 "$OUT/abc.log"; exit 2; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print('$v', d['ms_per_solve_median'], r['pass1_us_per_step'], r['kernels']['k_p2_spmv']['avg_launch_us_events'], r['kernels'].get('k_p1_spmv',{}).get('avg_launch_us_events'), d['config']['x_sha256_16'])" "$OUT/abc.log"
  done
done
