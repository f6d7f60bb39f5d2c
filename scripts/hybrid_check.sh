#!/bin/bash
# configs[4] (5M arcs, k = 500) on one GPU: the single-GPU solve vs the replicated-long-row
# partition over ONE RCCL rank (the N-independent per-step cost of the partition: rank
# totals, long-row epilogues, exchanges that move nothing), with rocprofv3 stats of the
# partitioned run.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 400 python bench.py --partition 1 --arcs 5000000 --steps 5 --warmup 1 > "$OUT/hybrid1_5m.log" 2>&1 || { tail -20 "$OUT/hybrid1_5m.log"; exit 3; }
tail -1 "$OUT/hybrid1_5m.log"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/hybrid_prof" -o run --output-format csv -- python3 "$ROOT/bench.py" --partition 1 --arcs 5000000 --steps 3 --warmup 1 --single-ref 0 > "$OUT/hybrid_prof.log" 2>&1 || { tail -20 "$OUT/hybrid_prof.log"; exit 4; }
python3 - "$OUT/hybrid_prof/run_kernel_stats.csv" <<'PY'
import csv, sys
for x in csv.DictReader(open(sys.argv[1])):
    print(x['Name'][:56].ljust(56), x['Calls'].rjust(6), '%.3f' % (float(x['AverageNs']) / 1000))
PY
