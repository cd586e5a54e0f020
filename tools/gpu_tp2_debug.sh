set -o pipefail
mkdir -p gpurun_out/tp
export HSA_ENABLE_IPC_MODE_LEGACY=0 BCG_AR_CAP_MB=512 BCG_STACKS_AFTER=45
timeout -k 10 240 python bench.py --gpus 2 --tp 2 --model qwen3-32b --sims-per-gpu 16 --max-batch-seqs 160 \
  --kv-cache-gb 12 --one-device --steps 2 --warmup 1 --fill-max-s 60 --deadline-s 1500 > gpurun_out/tp/tp2q.json 2> gpurun_out/tp/tp2q.err
echo rc=$?
grep -v "^\[W\|Gloo\|amdgpu.ids" gpurun_out/tp/tp2q.err | head -150
