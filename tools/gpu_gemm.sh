set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gemm_gpu.py > gpurun_out/gemm_test.log 2>&1; rc=$?
tail -15 gpurun_out/gemm_test.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u tools/tune_hand_gemm.py --m 64,128,256,448,768 --reps 10 --skip lm_head > gpurun_out/tune_hand.log 2>&1; rc=$?
cat gpurun_out/tune_hand.log | tail -40
exit $rc
