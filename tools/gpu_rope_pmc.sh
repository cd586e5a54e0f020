#!/bin/bash
# rope/decode tests, rope + decode-attention A/B (base vs new library), prefill-attention PMC (old vs new).
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
bash tools/gpu_decode_attn_ab.sh || exit 1
OUT=gpurun_out/pmc_old BCG_KERNELS_LIB=$PWD/build/libbcg_old.so NTS=4 bash tools/gpu_pmc_attn.sh || exit 1
OUT=gpurun_out/pmc_new NTS=4 bash tools/gpu_pmc_attn.sh || exit 1
