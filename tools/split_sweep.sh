export HSA_ENABLE_IPC_MODE_LEGACY=0; mkdir -p gpurun_out
for sp in 128 256 512 1024 2048; do echo "split=$sp"; BCG_BENCH_B=40,160 BCG_DECODE_SPLIT=$sp timeout -k 10 120 python tools/bench_ops.py --skip-gemm 2>&1 | grep '"ctx"' || exit 1; done
