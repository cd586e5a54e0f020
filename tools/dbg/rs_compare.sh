#!/bin/bash
# W4: reduce-scatter split-K (pp_w4) vs last-arriver (pp_w4nors) vs the committed kernel (pp_w4head),
# decode and prefill shapes (tools-only)
set -o pipefail
for round in 1 2; do
  for v in w4 w4nl w4nb w4nlnb w4head; do
    for s in "704 7168 5120 0 2" "704 7168 5120 0 3" "704 5120 5120 2 3" "704 5120 5120 2 4" "704 5120 17408 2 3" "704 5120 17408 2 4" "544 7168 5120 0 3" "1024 7168 5120 0 2" "1024 5120 17408 2 3" "704 34816 5120 1 1" "16384 7168 5120 0 1" "16384 34816 5120 1 1" "16384 5120 17408 2 1"; do
      [ -x build/pp_$v ] || continue
      timeout -k 5 60 build/pp_$v $s 20 || exit 1
    done
  done
done
