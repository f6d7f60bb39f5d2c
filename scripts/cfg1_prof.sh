#!/bin/bash
# configs[1] (50k arcs, two-pass k = 200, f = exp) alone under rocprofv3 --kernel-trace
# --stats, plus the bench line of the same workload; then the given pytest selection.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
cd "$ROOT"
if [ -n "${PYTEST_SEL:-}" ]; then
  timeout -k 10 600 python -u -m pytest $PYTEST_SEL -q -p no:cacheprovider --timeout 300 --timeout-method thread > "$OUT/pytest_sel.log" 2>&1
  rc=$?
  tail -8 "$OUT/pytest_sel.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
fi
timeout -k 10 300 python bench.py --headline-only 1 --arcs 50000 --k 200 --f exp --steps 20 > "$OUT/cfg1_bench.log" 2>&1 || { tail -20 "$OUT/cfg1_bench.log"; exit 3; }
tail -1 "$OUT/cfg1_bench.log"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/cfg1_prof" -o run --output-format csv -- python3 "$ROOT/bench.py" --headline-only 1 --arcs 50000 --k 200 --f exp --steps 5 > "$OUT/cfg1_prof.log" 2>&1 || { tail -20 "$OUT/cfg1_prof.log"; exit 4; }
python3 - "$OUT/cfg1_prof/run_kernel_stats.csv" <<'PY'
import csv, sys
for x in csv.DictReader(open(sys.argv[1])):
    print(x['Name'][:48].ljust(48), x['Calls'].rjust(6), '%.3f' % (float(x['AverageNs']) / 1000))
PY
