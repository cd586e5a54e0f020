set -o pipefail
mkdir -p gpurun_out
T=byzantine_consensus_llm_agents_amd/engine/tuned/tunableop_qwen3-14b_tp1.csv
grep -v "_16384_" $T > gpurun_out/base.csv
export PYTORCH_TUNABLEOP_ROTATING_BUFFER_SIZE=1024
timeout -k 10 400 python tools/tune_gemms.py --max-m 0 --extra-m 16384 --base gpurun_out/base.csv --out gpurun_out/retuned.csv > gpurun_out/retune.log 2>&1 || { tail -20 gpurun_out/retune.log; exit 1; }
tail -3 gpurun_out/retune.log
grep "_16384_" gpurun_out/retuned.csv
cp gpurun_out/retuned.csv $T
timeout -k 10 200 python tools/bench_prefill.py --m 16384 --modes default,tuned,rocblas --skip-attn > gpurun_out/prefill_gemm2.log 2>&1; rc=$?
grep -h "TF/s" gpurun_out/prefill_gemm2.log | grep -v attn
exit $rc
