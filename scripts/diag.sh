#!/bin/bash
# Dev diagnostics on the GPU box: stamp timeline of the SpMV-shaped launches
# (TPL_STAMP variant library) and PMC passes over scripts/pmc_drive.py.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/diag
mkdir -p "$OUT"
cd "$ROOT"
if [ "${STAMPS:-1}" = "1" ]; then
  TPL_LIB_PATH=$ROOT/two-pass-lanczos_amd/variants/libtpl_stamp.so timeout -k 10 240 python3 scripts/stamps.py > "$OUT/stamps.log" 2>&1 || { echo "stamps failed"; tail -20 "$OUT/stamps.log"; exit 2; }
  cat "$OUT/stamps.log"
fi
cd /tmp && export TMPDIR=/tmp
export TPL_NO_GRAPH=1
i=0
for group in "$@"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $group -d "$OUT/p$i" -o run --output-format csv -- python3 "$ROOT/scripts/pmc_drive.py" > "$OUT/p$i.log" 2>&1 || { echo "pass $i ($group) failed"; tail -5 "$OUT/p$i.log"; exit 3; }
done
python3 "$ROOT/scripts/pmc_summary.py" $(find "$OUT" -name '*counter_collection*' | sort) > "$OUT/summary.txt"
cat "$OUT/summary.txt"
