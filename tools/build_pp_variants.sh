#!/bin/bash
# Build one standalone timing binary per ping-pong GEMM variant (build/pp_<name>), on the CPU host.
#   tools/build_pp_variants.sh "name:-DFLAG -DFLAG2" ...
set -e
mkdir -p build
for spec in "$@"; do
  name=${spec%%:*}; flags=${spec#*:}
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fgpu-flush-denormals-to-zero -munsafe-fp-atomics \
    -Icsrc/kernels $flags -DVARIANT_NAME="\"$name\"" csrc/kernels/gemm_pp.hip csrc/bench/gemm_pp_bench.hip -o build/pp_$name &
done
wait
ls -la build/
