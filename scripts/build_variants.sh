#!/bin/bash
# Dev tool: build experiment variants of libtpl_amd.so into two-pass-lanczos_amd/variants/
# (one build dir each). Args: name=DEFINES (DEFINES: space-separated -D flags).
set -eu
ROOT=$(cd "$(dirname "$0")/.." && pwd)
CS=$ROOT/two-pass-lanczos_amd/csrc
mkdir -p "$ROOT/two-pass-lanczos_amd/variants"
base="-O3 -std=c++17 -fPIC -ffp-contract=off -Wall -Wno-unused-result -Wno-unused-value"
pids=()
for spec in "$@"; do
  name=${spec%%=*}; defs=${spec#*=}
  make -s -C "$CS" BUILD=build_$name OUT=../variants/libtpl_$name.so CXXFLAGS="$base $defs" > /tmp/build_$name.log 2>&1 &
  pids+=($!)
done
rc=0
for p in "${pids[@]}"; do wait $p || rc=1; done
ls -la "$ROOT/two-pass-lanczos_amd/variants"
exit $rc
