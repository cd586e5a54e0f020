#!/bin/bash
# Whole-library variant builds for A/B timing: build/libbcg_<name>.so, selected with BCG_KERNELS_LIB.
#   tools/build_kernel_variants.sh "name:-DFLAG ..." ...
set -e
mkdir -p build
# stamped with the tree's source hash (ops/hip.py refuses unstamped libraries); the -D flags are the variant
H=$(python -c "from byzantine_consensus_llm_agents_amd.utils.build import kernels_source_hash as h; print(h())")
for spec in "$@"; do
  name=${spec%%:*}; flags=${spec#*:}
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -shared -fPIC -fgpu-flush-denormals-to-zero \
    -munsafe-fp-atomics -Icsrc/kernels -DBCG_SOURCE_HASH=\"$H\" $flags csrc/kernels/*.hip -o build/libbcg_$name.so &
done
wait
ls build
