#!/bin/bash
# W4 split-K vs stream-K (split 0) over decode-size shapes (tools-only sweep)
set -o pipefail
mkdir -p gpurun_out/sk
for round in 1 2; do
  for M in 544 704 1024; do
    for s in "7168 5120 0" "5120 5120 2" "34816 5120 1" "5120 17408 2"; do
      set -- $s
      for sp in 0 1 2 3 4; do
        timeout -k 5 60 build/pp_w4 $M $1 $2 $3 $sp 30 || exit 1
      done
    done
  done
done | tee gpurun_out/sk/sweep.jsonl
