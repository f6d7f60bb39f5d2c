#!/bin/bash
# Round-6 checkpoint on one GPU: the GPU suite, a stamp timeline (abvar/libtpl_stamp.so),
# the full default bench line, the headline's rank shares (scripts/rank_share.py --arcs
# 500000) and an A/B of the in-tree library against abvar/ variants named as arguments.
# Stops at the first failure.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/${TAG:-r06}
mkdir -p "$OUT" "$ROOT/gpurun_out/diag"
cd "$ROOT"
if [ "${SKIP_TESTS:-0}" != "1" ]; then
  echo "== pytest -m gpu"
  timeout -k 10 500 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
  rc=$?; tail -2 "$OUT/pytest_gpu.log"
  [ $rc -ne 0 ] && { echo "pytest rc=$rc"; tail -30 "$OUT/pytest_gpu.log"; exit 1; }
fi
if [ "${SKIP_STAMPS:-0}" != "1" ]; then
  echo "== stamps"
  TPL_LIB_PATH=$ROOT/abvar/libtpl_stamp.so timeout -k 10 240 python3 scripts/stamps.py > "$OUT/stamps.log" 2>&1 || { echo "stamps failed"; tail -20 "$OUT/stamps.log"; exit 2; }
  cp "$ROOT/gpurun_out/diag/pass1_stamps.npz" "$OUT/"
fi
if [ "${SKIP_BENCH:-0}" != "1" ]; then
  echo "== bench (default)"
  timeout -k 10 600 python bench.py > "$OUT/bench.log" 2>&1 || { echo "bench failed"; tail -20 "$OUT/bench.log"; exit 3; }
  tail -1 "$OUT/bench.log" | cut -c1-400
fi
if [ "${SHARES:-1}" = "1" ]; then
  echo "== rank shares, 500k"
  timeout -k 10 500 python scripts/rank_share.py --arcs 500000 --out "$OUT/rank_share_500k.json" > "$OUT/rank_share_500k.log" 2>&1 || { echo "rank_share failed"; tail -20 "$OUT/rank_share_500k.log"; exit 4; }
  tail -4 "$OUT/rank_share_500k.log" | cut -c1-300
fi
if [ $# -gt 0 ]; then
  echo "== A/B: in-tree vs $*"
  REPS=${REPS:-3} VDIR=abvar timeout -k 10 900 bash scripts/ab_bench.sh "$@" > "$OUT/ab.txt" 2>&1 || { echo "ab failed"; tail -20 "$OUT/ab.txt"; exit 5; }
  cat "$OUT/ab.txt"
fi
