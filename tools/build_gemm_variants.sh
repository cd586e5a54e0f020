#!/bin/bash
# Build one standalone timing binary per 256x256 GEMM variant (build/pp_<name>), on the CPU host.
#   tools/build_gemm_variants.sh "name:SRC:-DFLAG -DFLAG2" ...   SRC = pp | rs
set -e
mkdir -p build
for spec in "$@"; do
  name=${spec%%:*}; rest=${spec#*:}; src=${rest%%:*}; flags=${rest#*:}
  fn=bcg_gemm_$src
  file=csrc/kernels/gemm_$src.hip; [ -f $file ] || file=csrc/experimental/gemm_$src.hip
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fgpu-flush-denormals-to-zero -munsafe-fp-atomics \
    -Icsrc/kernels $flags -DGEMM_FN=$fn -DVARIANT_NAME="\"$name\"" $file csrc/bench/gemm_pp_bench.hip \
    -o build/pp_$name &
done
wait
ls build/
