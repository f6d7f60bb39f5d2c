#!/bin/bash
# Round-5 GPU session on the final tree: parity tests, bench, rocprofv3 kernel trace +
# stats and the two PMC passes of the headline, the rank shares (prediction) and one RCCL
# rank at 5M beside the single-GPU solve. Stops at the first failure.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out
cd "$ROOT"
SKIP_PMC=0 bash scripts/r05_check.sh || exit $?
echo "== rank shares"
timeout -k 10 500 python scripts/rank_share.py > "$OUT/rank_share.log" 2>&1 || { echo "rank_share failed"; tail -20 "$OUT/rank_share.log"; exit 6; }
tail -4 "$OUT/rank_share.log" | cut -c1-300
echo "== one RCCL rank at 5M vs one GPU"
timeout -k 10 400 python bench.py --gpus 1 --partition 1 --steps 5 --warmup 1 > "$OUT/rep1_bench.log" 2>&1 || { echo "rep1 bench failed"; tail -20 "$OUT/rep1_bench.log"; exit 7; }
tail -1 "$OUT/rep1_bench.log" | cut -c1-300
