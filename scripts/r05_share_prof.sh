#!/bin/bash
# Round 5: per-kernel times of rank 0's share of the replicated partition at N (default 8),
# solved as a one-rank partition (scripts/rank_share.py --single 0) under rocprofv3
# --kernel-trace --stats: the kernels one rank runs per step, for the `predicted` block.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out
N=${N:-8}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d "$OUT/prof_share$N" -o run --output-format csv -- python3 "$ROOT/scripts/rank_share.py" --ranks $N --all-ranks 0 --single 0 --reps 3 --out "$OUT/rank_share_prof$N.json" > "$OUT/share_prof$N.log" 2>&1 || { echo "share prof failed"; tail -20 "$OUT/share_prof$N.log"; exit 2; }
T=$(find "$OUT/prof_share$N" -name '*kernel_trace.csv' | head -1)
S=$(find "$OUT/prof_share$N" -name '*kernel_stats.csv' | head -1)
cp "$T" "$OUT/prof_share$N/run_kernel_trace.csv" 2>/dev/null; cp "$S" "$OUT/prof_share$N/run_kernel_stats.csv" 2>/dev/null
python3 "$ROOT/scripts/kernel_medians.py" "$OUT/prof_share$N/run_kernel_trace.csv" "$OUT/share_medians$N.json" > "$OUT/share_medians$N.txt"
cut -d, -f1-5 "$OUT/prof_share$N/run_kernel_stats.csv" | head -14
head -20 "$OUT/share_medians$N.txt"
