#!/bin/bash
# Whole-library variant builds for A/B timing: build/libbcg_<name>.so, selected with BCG_KERNELS_LIB.
#   tools/build_kernel_variants.sh "name:-DFLAG ..." ...
set -e
mkdir -p build
for spec in "$@"; do
  name=${spec%%:*}; flags=${spec#*:}
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -shared -fPIC -fgpu-flush-denormals-to-zero \
    -munsafe-fp-atomics -Icsrc/kernels $flags csrc/kernels/*.hip -o build/libbcg_$name.so &
done
wait
ls build
