#!/bin/bash
# The reference's accuracy / orthogonality experiments for f = exp (src/bin/stability.rs,
# src/bin/orthogonality.rs) on the engine — the two-pass solves now evaluate exp(T_k) e_1
# on the device (k_ftk_exp) — compared with the published CSVs.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/r03_harness
mkdir -p "$OUT"
cd "$ROOT/two-pass-lanczos_amd"
for sc in well-conditioned ill-conditioned; do
  for exp in accuracy orthogonality; do
    timeout -k 10 300 python -m tpl_amd.harness $exp --function exp --scenario $sc \
      --output "$OUT/${exp}_exp_${sc}.csv" > "$OUT/${exp}_exp_${sc}.log" 2>&1 || { echo "$exp $sc failed"; tail -5 "$OUT/${exp}_exp_${sc}.log"; exit 3; }
  done
done
python3 "$ROOT/scripts/compare_harness.py" "$OUT" | tee "$OUT/COMPARE.txt"
