#!/bin/bash
# A/B: SpMV slot batch (PNP_SPMV_BATCH 1 / 2 / 4)
set -u
OUT=gpurun_out/$1; mkdir -p "$OUT"; : > "$OUT/ab_spmv.log"
for i in 1 2 3; do
  for b in 1 2 4; do
    echo -n "batch=$b " >> "$OUT/ab_spmv.log"
    PNP_SPMV_BATCH=$b timeout -k 10 120 python tools/ab_asm.py >> "$OUT/ab_spmv.log" 2>&1 || exit $?
  done
done
