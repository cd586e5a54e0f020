set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_gpu.py tests/test_kernels_gpu.py -m gpu > gpurun_out/t.log 2>&1 || { tail -30 gpurun_out/t.log; exit 1; }
tail -2 gpurun_out/t.log
bash tools/gpu_tune_hand.sh || exit 1
cp gpurun_out/hand_gemm_qwen3-14b.json byzantine_consensus_llm_agents_amd/engine/tuned/hand_gemm.json
bash tools/gpu_bench.sh
