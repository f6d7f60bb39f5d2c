#!/bin/bash
# rocprofv3 PMC passes over scripts/pmc_drive.py (dev tool). One counter group per pass.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/pmc
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
export TPL_NO_GRAPH=1
i=0
for group in "$@"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $group -d "$OUT/p$i" -o run --output-format csv -- python3 "$ROOT/scripts/pmc_drive.py" > "$OUT/p$i.log" 2>&1 || { echo "pass $i failed"; tail -5 "$OUT/p$i.log"; exit 1; }
done
find "$OUT" -name '*counter_collection*' | sort > "$OUT/files.txt"
python3 "$ROOT/scripts/pmc_summary.py" $(cat "$OUT/files.txt") > "$OUT/summary.txt"
cat "$OUT/summary.txt"
