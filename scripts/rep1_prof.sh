#!/bin/bash
# Dev tool (GPU box): the replicated-long-row partition over ONE RCCL rank at configs[4]'s
# 5M arcs — bench line with the single-GPU solve of the same workload beside it, then a
# rocprofv3 kernel trace of the partitioned solves alone (per-kernel cost of the
# partition's own launches: rank totals, long-row epilogues, RCCL).
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 400 python bench.py --gpus 1 --partition 1 --steps 5 --warmup 1 --parity 0 \
  > "$OUT/rep1_bench.log" 2>&1 || { echo "rep1 bench failed"; tail -20 "$OUT/rep1_bench.log"; exit 2; }
tail -1 "$OUT/rep1_bench.log"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/prof_rep1" -o run --output-format csv -- \
  python3 "$ROOT/bench.py" --gpus 1 --partition 1 --steps 3 --warmup 1 --parity 0 --single-ref 0 \
  > "$OUT/rep1_prof.log" 2>&1 || { echo "rep1 rocprof failed"; tail -20 "$OUT/rep1_prof.log"; exit 3; }
find "$OUT/prof_rep1" -name '*kernel_stats*' -exec head -14 {} \;
