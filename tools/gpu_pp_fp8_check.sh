set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_gpu.py -m gpu -k "pp" > gpurun_out/pp_tests.log 2>&1 || { tail -30 gpurun_out/pp_tests.log; exit 1; }
tail -1 gpurun_out/pp_tests.log
timeout -k 10 300 python -u tools/bench_fp8_gemm.py --ms 8192,16384 > gpurun_out/fp8_prefill.log 2>&1 || { tail -20 gpurun_out/fp8_prefill.log; exit 1; }
cat gpurun_out/fp8_prefill.log
