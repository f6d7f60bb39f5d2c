#!/bin/bash
# Dev tool: build an experiment variant of libtpl_amd.so from an EDITED COPY of the
# sources (the product sources carry no experiment switches). Usage:
#   scripts/build_variant_src.sh NAME EDIT.py [EXTRA_CXXFLAGS]
# EDIT.py runs with the copy's csrc directory as its working directory and edits the files
# there; the library lands in two-pass-lanczos_amd/variants/libtpl_NAME.so and the
# kernel resource usage (VGPRs, occupancy, spills) in /tmp/tplvar_NAME/usage.txt.
set -eu
ROOT=$(cd "$(dirname "$0")/.." && pwd)
name=$1; edit=$(cd "$(dirname "$2")" && pwd)/$(basename "$2"); extra=${3:-}
W=/tmp/tplvar_$name
rm -rf "$W"; mkdir -p "$W/two-pass-lanczos_amd" "$W/include"
cp -r "$ROOT/two-pass-lanczos_amd/csrc" "$W/two-pass-lanczos_amd/"
rm -rf "$W/two-pass-lanczos_amd/csrc/build"
cp "$ROOT/include/"*.h "$W/include/"
(cd "$W/two-pass-lanczos_amd/csrc" && python3 "$edit")
mkdir -p "$ROOT/two-pass-lanczos_amd/variants"
base="-O3 -std=c++17 -fPIC -ffp-contract=off -Wall -Wno-unused-result -Wno-unused-value"
make -s -C "$W/two-pass-lanczos_amd/csrc" OUT="$ROOT/two-pass-lanczos_amd/variants/libtpl_$name.so" \
     CXXFLAGS="$base $extra" > "$W/build.log" 2>&1 || { tail -30 "$W/build.log"; exit 1; }
(cd "$W/two-pass-lanczos_amd/csrc" && /opt/rocm/bin/hipcc $base $extra --offload-arch=gfx950 \
   -munsafe-fp-atomics --cuda-device-only -c tpl_kernels.hip -o /dev/null \
   -Rpass-analysis=kernel-resource-usage 2>&1 |
   grep -A8 "Function Name: _ZN3tpl9k_p[12]_\(spmv\|axpy\)ILi\(58\|12\)E" |
   grep -E "Function Name|VGPRs|Occupancy|Spill" > "$W/usage.txt") || true
echo "built variants/libtpl_$name.so"; cat "$W/usage.txt" | sed 's/.*remark: *//'
