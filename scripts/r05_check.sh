#!/bin/bash
# Round-5 GPU session: parity tests, bench, rocprofv3 kernel trace + stats of the
# headline, and the kernel-boundary analysis of that trace. Stops at the first failure.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
cd "$ROOT"
if [ "${SKIP_TESTS:-0}" != "1" ]; then
  echo "== pytest -m gpu"
  timeout -k 10 ${TEST_TIMEOUT:-600} python -u -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 120 --timeout-method thread ${PYTEST_ARGS:-} > "$OUT/pytest_gpu.log" 2>&1 || { echo "pytest failed rc=$?"; tail -30 "$OUT/pytest_gpu.log"; exit 2; }
  tail -2 "$OUT/pytest_gpu.log"
fi
echo "== bench"
timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > "$OUT/bench.log" 2>&1 || { echo "bench failed"; tail -20 "$OUT/bench.log"; exit 3; }
tail -1 "$OUT/bench.log" | cut -c1-600
[ "${SKIP_PROF:-0}" = "1" ] && exit 0
echo "== rocprofv3 kernel trace"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python3 "$ROOT/bench.py" --steps 5 --warmup 1 --headline-only 1 > "$OUT/prof.log" 2>&1 || { echo "rocprof failed"; tail -20 "$OUT/prof.log"; exit 4; }
T=$(find "$OUT/prof" -name '*kernel_trace.csv' | head -1)
S=$(find "$OUT/prof" -name '*kernel_stats.csv' | head -1)
cp "$T" "$OUT/prof/run_kernel_trace.csv" 2>/dev/null; cp "$S" "$OUT/prof/run_kernel_stats.csv" 2>/dev/null
python3 "$ROOT/scripts/trace_gaps.py" "$OUT/prof/run_kernel_trace.csv" > "$OUT/gaps.txt"
python3 "$ROOT/scripts/kernel_medians.py" "$OUT/prof/run_kernel_trace.csv" > "$OUT/medians.txt"
head -12 "$OUT/gaps.txt"; head -6 "$OUT/medians.txt"
tail -1 "$OUT/prof.log" | cut -c1-300
[ "${SKIP_PMC:-1}" = "1" ] && exit 0
echo "== rocprofv3 PMC (FETCH_SIZE, WRITE_SIZE: separate passes)"
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $c -d "$OUT/pmc_$c" -o run --output-format csv -- python3 "$ROOT/bench.py" --steps 1 --warmup 0 --headline-only 1 > "$OUT/pmc_$c.log" 2>&1 || { echo "pmc $c failed"; tail -5 "$OUT/pmc_$c.log"; exit 5; }
done
python3 "$ROOT/scripts/pmc_summary.py" $(find "$OUT" -path '*pmc_*' -name '*counter_collection*') > "$OUT/pmc_summary.txt"
cat "$OUT/pmc_summary.txt"
