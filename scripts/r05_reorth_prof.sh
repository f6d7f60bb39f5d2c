#!/bin/bash
# Round-5: per-kernel rocprofv3 stats of the CGS2 one-pass solve (configs[3]) and the
# driver-equivalent bench command.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/bench_driver.log" 2>&1 || { echo "bench failed"; tail -20 "$OUT/bench_driver.log"; exit 2; }
tail -c 300 "$OUT/bench_driver.log"; echo
cd /tmp && export TMPDIR=/tmp
REPS=1 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/prof_reorth" -o run --output-format csv -- python3 "$ROOT/scripts/reorth_bench.py" > "$OUT/reorth_prof.log" 2>&1 || { echo "reorth prof failed"; tail -20 "$OUT/reorth_prof.log"; exit 3; }
S=$(find "$OUT/prof_reorth" -name '*kernel_stats.csv' | head -1)
cut -d, -f1-5 "$S" | head -12
grep '^{' "$OUT/reorth_prof.log"
