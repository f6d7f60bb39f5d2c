#!/bin/bash
# Build ablation variants of libtpl_amd.so into scripts/ablate/ (experiments only).
set -e
cd "$(dirname "$0")/../two-pass-lanczos_amd/csrc"
mkdir -p ../../scripts/ablate
# args: NAME=DEFINES... e.g. ab1="-DTPL_ABLATE=1" c256="-DTPL_CHUNK_ROWS=256"
for spec in "$@"; do
  A=${spec%%=*}; DEFS=${spec#*=}
  rm -rf build_ab$A && mkdir -p build_ab$A
  for f in tpl_kernels tpl_push; do /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -ffp-contract=off --offload-arch=gfx950 $DEFS -c $f.hip -o build_ab$A/$f.o; done
  for f in tpl_runtime tpl_ftk tpl_loader; do /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -ffp-contract=off $DEFS -c $f.cpp -o build_ab$A/$f.o; done
  /opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o ../../scripts/ablate/libtpl_amd_ab$A.so build_ab$A/*.o -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
  rm -rf build_ab$A
done
