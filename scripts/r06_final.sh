#!/bin/bash
# Round-6 GPU session on a candidate final tree: parity tests, bench, rocprofv3 kernel
# trace + stats and the two PMC passes of the headline (scripts/gpu_check.sh), then the
# rank shares of both partitioned workloads (the N > 1 lines' predictions) and the N = 2
# rehearsal over the host transport. Stops at the first failure.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out
cd "$ROOT"
bash scripts/gpu_check.sh || exit $?
echo "== rank shares (headline, 500k)"
timeout -k 10 500 python scripts/rank_share.py --arcs 500000 --out "$OUT/rank_share_500k.json" > "$OUT/rank_share_500k.log" 2>&1 || { echo "rank_share 500k failed"; tail -20 "$OUT/rank_share_500k.log"; exit 6; }
tail -4 "$OUT/rank_share_500k.log" | cut -c1-200
if [ "${SHARES_5M:-1}" = "1" ]; then
  echo "== rank shares (configs[4], 5M)"
  timeout -k 10 600 python scripts/rank_share.py --out "$OUT/rank_share.json" > "$OUT/rank_share.log" 2>&1 || { echo "rank_share 5M failed"; tail -20 "$OUT/rank_share.log"; exit 7; }
  tail -4 "$OUT/rank_share.log" | cut -c1-200
fi
echo "== rehearsal: bench.py --gpus 2, both ranks on GPU 0, host transport"
TPL_DEVICE=0 TPL_DIST_TRANSPORT=host timeout -k 10 700 python bench.py --gpus 2 --steps 3 --warmup 1 --child-timeout 650 > "$OUT/reh2.log" 2>&1 || { echo "rehearsal failed"; tail -20 "$OUT/reh2.log"; exit 8; }
tail -1 "$OUT/reh2.log" | cut -c1-300
