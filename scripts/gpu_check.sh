#!/bin/bash
# One GPU session: parity tests, bench, rocprofv3 kernel stats. Stops at the first
# GPU fault / abort / timeout (exit codes other than 0 and 1 from pytest).
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
cd "$ROOT"
echo "== pytest -m gpu"
timeout -k 10 ${TEST_TIMEOUT:-900} python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread ${PYTEST_ARGS:-} > "$OUT/pytest_gpu.log" 2>&1
rc=$?
tail -5 "$OUT/pytest_gpu.log"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
[ "${SKIP_BENCH:-0}" = "1" ] && exit $rc
echo "== bench"
timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > "$OUT/bench.log" 2>&1 || { echo "bench failed"; tail -20 "$OUT/bench.log"; exit 3; }
tail -2 "$OUT/bench.log"
[ "${SKIP_PROF:-0}" = "1" ] && exit $rc
echo "== rocprofv3 kernel trace"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python3 "$ROOT/bench.py" --steps 5 --warmup 1 --headline-only 1 > "$OUT/prof.log" 2>&1 || { echo "rocprof failed"; tail -20 "$OUT/prof.log"; exit 4; }
find "$OUT/prof" -name '*stats*' | head
[ "${SKIP_PMC:-0}" = "1" ] && exit $rc
echo "== rocprofv3 PMC (FETCH_SIZE, WRITE_SIZE: separate passes)"
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 600 rocprofv3 --pmc $c -d "$OUT/pmc_$c" -o run --output-format csv -- python3 "$ROOT/bench.py" --steps 1 --warmup 0 --headline-only 1 > "$OUT/pmc_$c.log" 2>&1 || { echo "pmc $c failed"; tail -5 "$OUT/pmc_$c.log"; exit 5; }
done
python3 "$ROOT/scripts/pmc_summary.py" $(find "$OUT" -path '*pmc_*' -name '*counter_collection*') > "$OUT/pmc_summary.txt"
cat "$OUT/pmc_summary.txt"
exit $rc
