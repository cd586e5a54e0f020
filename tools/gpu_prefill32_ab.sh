#!/bin/bash
# Prefill attention A/B on one GPU: the prefill kernel tests, then tools/bench_prefill.py for the
# shipped library and every build/libbcg_p32_*.so variant (tools/build_kernel_variants.sh), and one
# rocprofv3 counter pass over the 32x32 kernel.  Output: gpurun_out/p32v/.
set -o pipefail
mkdir -p gpurun_out/p32v
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "prefill" -x -q --timeout 120 \
  --timeout-method thread > gpurun_out/p32v/tests.log 2>&1 || { tail -30 gpurun_out/p32v/tests.log; exit 1; }
tail -2 gpurun_out/p32v/tests.log
SHAPES=${SHAPES:-12x1024+512,16x900+400,8x2048+0,16x1000+380}
for v in base $(ls build 2>/dev/null | grep '^libbcg_p32_' | sed 's/^libbcg_p32_//; s/\.so$//') base; do
  if [ $v = base ]; then lib=byzantine_consensus_llm_agents_amd/ops/libbcg_kernels.so; else lib=build/libbcg_p32_$v.so; fi
  echo "== $v" >> gpurun_out/p32v/all.log
  BCG_KERNELS_LIB=$lib timeout -k 10 150 python -u tools/bench_prefill.py --skip-gemm --tile-rows ${ROWS:-64,128,256} \
    --attn-shapes $SHAPES >> gpurun_out/p32v/all.log 2>&1 || exit 1
done
TAG=p32 LIMIT=120 bash tools/gpu_run.sh pmc prefill_attn32 SQ_WAVES,SQ_WAVE_CYCLES,SQ_BUSY_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_LDS,SQ_INSTS_MFMA,SQ_VALU_MFMA_BUSY_CYCLES,SQ_INSTS_VALU \
  -- python tools/bench_prefill.py --skip-gemm --tile-rows 128 --attn-shapes 16x1000+380 > gpurun_out/p32v/pmc.log 2>&1
grep -v amdgpu.ids gpurun_out/p32v/all.log; tail -12 gpurun_out/p32v/pmc.log
