#!/bin/bash
# Tune the M=16384 prefill-chunk GEMMs over rocBLAS solutions only, splice the
# qkv/o entries into a copy of the shipped table, and time default vs spliced.
set -o pipefail
mkdir -p gpurun_out
T=byzantine_consensus_llm_agents_amd/engine/tuned/tunableop_qwen3-14b_tp1.csv
grep -v "_16384_" $T > gpurun_out/base.csv
export PYTORCH_TUNABLEOP_HIPBLASLT_ENABLED=0
timeout -k 10 400 python tools/tune_gemms.py --max-m 0 --extra-m 16384 --base gpurun_out/base.csv --out gpurun_out/rocblas16k.csv > gpurun_out/retune_rb.log 2>&1 || { tail -20 gpurun_out/retune_rb.log; exit 1; }
unset PYTORCH_TUNABLEOP_HIPBLASLT_ENABLED
grep "_16384_" gpurun_out/rocblas16k.csv
cp $T gpurun_out/spliced.csv
sed -i -e "/tn_7168_16384_5120/d" -e "/tn_5120_16384_5120_ld_5120_5120_5120/d" gpurun_out/spliced.csv
grep -E "tn_7168_16384_5120|tn_5120_16384_5120_ld_5120_5120_5120" gpurun_out/rocblas16k.csv >> gpurun_out/spliced.csv
cp gpurun_out/spliced.csv $T
timeout -k 10 200 python tools/bench_prefill.py --m 16384 --modes default,tuned --skip-attn > gpurun_out/prefill_gemm3.log 2>&1; rc=$?
grep -h "TF/s" gpurun_out/prefill_gemm3.log
exit $rc
