#!/bin/bash
# Round-5 GPU session: the replicated partition's per-rank share at N = 8/4/2/1 through one
# RCCL rank (scripts/rank_share.py), one RCCL rank at 5M against the single-GPU solve
# (the beta rank total folded into k_p1_axpy), and the device-vs-host inv at k = 1000-1365.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
cd "$ROOT"
echo "== rank shares"
timeout -k 10 500 python scripts/rank_share.py > "$OUT/rank_share.log" 2>&1 || { echo "rank_share failed"; tail -20 "$OUT/rank_share.log"; exit 2; }
tail -4 "$OUT/rank_share.log" | cut -c1-400
echo "== one RCCL rank at 5M vs one GPU"
timeout -k 10 400 python bench.py --gpus 1 --partition 1 --steps 5 --warmup 1 > "$OUT/rep1_bench.log" 2>&1 || { echo "rep1 bench failed"; tail -20 "$OUT/rep1_bench.log"; exit 3; }
tail -1 "$OUT/rep1_bench.log" | cut -c1-300
echo "== device vs host inv, large k"
timeout -k 10 300 python scripts/ftk_timing.py 5000:1000 5000:1365 50000:1000 50000:1365 > "$OUT/ftk_timing.log" 2>&1 || { echo "ftk timing failed"; tail -20 "$OUT/ftk_timing.log"; exit 4; }
cat "$OUT/ftk_timing.log"
