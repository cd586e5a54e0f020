#!/bin/bash
# split-K tail cost at decode sizes: full kernel vs no tail vs stores-only (tools-only)
set -o pipefail
for round in 1 2; do
  for v in w4 w4t1 w4t2; do
    for s in "704 7168 5120 0 3" "704 5120 5120 2 3" "704 5120 17408 2 4" "704 7168 5120 0 2" "704 7168 5120 0 1"; do
      timeout -k 5 60 build/pp_$v $s 30 || exit 1
    done
  done
done
