#!/bin/bash
# Dev tool: bench.py's headline numbers (pass one per step, isolated kernels) for each
# experiment variant library (two-pass-lanczos_amd/variants/libtpl_<name>.so).
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
for name in "$@"; do
  TPL_LIB_PATH=$ROOT/two-pass-lanczos_amd/variants/libtpl_$name.so timeout -k 10 200 python bench.py --one-pass 0 --other-configs 0 --cpu-baseline 0 --pcie 0 --steps 5 > /tmp/bv.log 2>&1 || { echo "$name failed"; tail -5 /tmp/bv.log; exit 1; }
  python - "$name" <<'PY'
import json, sys
d = json.loads(open("/tmp/bv.log").read().strip().splitlines()[-1])
r = d.get("roofline_live", d["roofline"])
print(json.dumps({"variant": sys.argv[1], "ms": d["ms_per_step"], "p1_step": r["pass1_us_per_step"], "p2_live": r["avg_launch_us_events"], **r["kernels_us_isolated"]}))
PY
done
