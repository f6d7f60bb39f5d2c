#!/bin/bash
# Round-6 GPU session: the GPU suite on the in-tree library, a stamp timeline of the
# stamp build (abvar/libtpl_stamp.so), then the headline bench alternated between the
# in-tree library and the abvar/ variants named as arguments. Stops at the first failure.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/${TAG:-r06}
mkdir -p "$OUT" "$ROOT/gpurun_out/diag"
cd "$ROOT"
if [ "${SKIP_TESTS:-0}" != "1" ]; then
  echo "== pytest -m gpu"
  timeout -k 10 ${TEST_TIMEOUT:-500} python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread ${PYTEST_ARGS:-} > "$OUT/pytest_gpu.log" 2>&1
  rc=$?
  tail -3 "$OUT/pytest_gpu.log"
  [ $rc -ne 0 ] && { echo "pytest rc=$rc"; tail -30 "$OUT/pytest_gpu.log"; exit 1; }
fi
if [ "${SKIP_STAMPS:-0}" != "1" ]; then
  echo "== stamps"
  TPL_LIB_PATH=$ROOT/abvar/libtpl_stamp.so timeout -k 10 240 python3 scripts/stamps.py > "$OUT/stamps.log" 2>&1 || { echo "stamps failed"; tail -20 "$OUT/stamps.log"; exit 2; }
  cp "$ROOT/gpurun_out/diag/pass1_stamps.npz" "$OUT/" 2>/dev/null
  grep -A12 "pass-one step" "$OUT/stamps.log" | head -14
fi
if [ $# -gt 0 ]; then
  echo "== A/B: in-tree vs $*"
  REPS=${REPS:-3} VDIR=abvar timeout -k 10 ${AB_TIMEOUT:-900} bash scripts/ab_bench.sh "$@" > "$OUT/ab.txt" 2>&1 || { echo "ab failed"; tail -20 "$OUT/ab.txt"; exit 3; }
  cat "$OUT/ab.txt"
fi
if [ "${REH:-0}" = "1" ]; then
  echo "== rehearsal: bench.py --gpus 2, both ranks on GPU 0, host transport"
  TPL_DEVICE=0 TPL_DIST_TRANSPORT=host timeout -k 10 700 python bench.py --gpus 2 --steps 3 --warmup 1 --child-timeout 650 > "$OUT/reh2.log" 2>&1 || { echo "rehearsal failed"; tail -20 "$OUT/reh2.log"; exit 4; }
  tail -1 "$OUT/reh2.log" | cut -c1-600
fi
