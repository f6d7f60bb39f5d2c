#!/bin/bash
# Round 5: the reference's tradeoff (500k arcs, k = 50..1000) and scalability (5k / 50k /
# 500k arcs, k = 500) experiments on the MI355X engine (tpl_amd.harness), CSVs into
# gpurun_out/harness/.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/harness
mkdir -p "$OUT"
cd "$ROOT/two-pass-lanczos_amd"
timeout -k 10 600 python -m tpl_amd.harness tradeoff --arcs 500000 --output "$OUT/tradeoff_arcs500k.csv" > "$OUT/tradeoff.log" 2>&1 || { echo "tradeoff failed"; tail -20 "$OUT/tradeoff.log"; exit 2; }
timeout -k 10 600 python -m tpl_amd.harness scalability --arcs 50000 100000 150000 200000 250000 300000 350000 400000 450000 500000 --output "$OUT/scalability_k500.csv" > "$OUT/scalability.log" 2>&1 || { echo "scalability failed"; tail -20 "$OUT/scalability.log"; exit 3; }
cat "$OUT/tradeoff_arcs500k.csv" "$OUT/scalability_k500.csv"
