#!/bin/bash
# Round-6 A/B of environment settings (scripts/env_ab.sh), alternated REPS times. Each
# argument is one variant's "NAME=VALUE ..." list; "@/" stands for the repo root on the box
# (e.g. "TPL_LIB_PATH=@/abvar/libtpl_lab.so TPL_BIN_BALANCE=2").
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/${TAG:-r06}
mkdir -p "$OUT"
cd "$ROOT"
vs=()
for v in "$@"; do vs+=("${v//@\//$ROOT/}"); done
REPS=${REPS:-3} timeout -k 10 ${AB_TIMEOUT:-1000} bash scripts/env_ab.sh "${vs[@]}" > "$OUT/env_ab.txt" 2>&1 || { echo "env ab failed"; tail -20 "$OUT/env_ab.txt"; exit 3; }
sed "s#$ROOT/##g" "$OUT/env_ab.txt"
