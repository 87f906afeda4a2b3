#!/bin/bash
# A/B: non-temporal loads of the SpMV values (PNP_SPMV_NT)
set -u
OUT=gpurun_out/$1; mkdir -p "$OUT"; : > "$OUT/ab_spmv_nt.log"
for i in 1 2 3; do
  for nt in 0 1; do
    echo -n "nt=$nt " >> "$OUT/ab_spmv_nt.log"
    PNP_SPMV_NT=$nt timeout -k 10 120 python tools/ab_asm.py >> "$OUT/ab_spmv_nt.log" 2>&1 || exit $?
  done
done
