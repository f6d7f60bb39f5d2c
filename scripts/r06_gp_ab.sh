#!/bin/bash
# Round-6 A/B of the replicated partition's gathered norm partials: the
# headline's rank shares at N = 8 and 2 (scripts/rank_share.py: each share solved on one
# GPU through one RCCL rank) with the in-tree library and with abvar/libtpl_nogp.so (the
# rank-total launch), alternated REPS times; then configs[4]'s N = 8 share the same way.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/${TAG:-r06gp}
mkdir -p "$OUT"
cd "$ROOT"
for arcs in 500000 5000000; do
  for rep in $(seq 1 ${REPS:-3}); do
    for v in tree nogp; do
      if [ "$v" = tree ]; then lib=""; else lib="TPL_LIB_PATH=$ROOT/abvar/libtpl_$v.so"; fi
      env $lib timeout -k 10 300 python scripts/rank_share.py --arcs $arcs --ranks 8 2 --all-ranks 0 --single 0 --reps 5 --out "$OUT/share_${arcs}_${v}_$rep.json" > "$OUT/share_${arcs}_${v}_$rep.log" 2>&1 || { echo "rank_share $arcs $v failed"; tail -20 "$OUT/share_${arcs}_${v}_$rep.log"; exit 2; }
      python3 -c "
import json,sys; d=json.load(open(sys.argv[1]))
print(sys.argv[2], sys.argv[3], ' '.join(f\"N{n}: {s['one_rank_replicated']['ms_per_solve']} ms p1 {s['one_rank_replicated']['pass1_us_per_step']} p2 {s['one_rank_replicated']['pass2_us_per_step']}\" for n, s in d['shares'].items()))" "$OUT/share_${arcs}_${v}_$rep.json" $arcs $v
    done
  done
done
