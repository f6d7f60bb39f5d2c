#!/bin/bash
# Dev check: the 5M one-GPU leg's time with and without the bench's earlier legs in the
# same process (does a previous leg slow it?).
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"; mkdir -p gpurun_out
for args in "--one-pass 0 --pcie 0 --other-configs 0" "--pcie 0 --other-configs 0" "--one-pass 0 --pcie 0" "--one-pass 0 --other-configs 0"; do
  out=$(timeout -k 10 400 python bench.py --cpu-baseline 0 $args 2>/dev/null | grep '^{' | tail -1)
  python3 -c "import json,sys; d=json.loads(sys.argv[1]); c=d['configs4_5m_1gpu']; print('$args', '|', c['ms_per_solve'], c['ms_per_solve_each'], c['k_p2_spmv_us'])" "$out"
done
