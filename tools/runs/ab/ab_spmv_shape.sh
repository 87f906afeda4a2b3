#!/bin/bash
# A/B: SpMV shape (PNP_SPMV_LPR x PNP_SPMV_BATCH), interleaved, plus the solver GPU tests at LPR=2
set -u
OUT=gpurun_out/$1; mkdir -p "$OUT"; : > "$OUT/ab_spmv_shape.log"
for i in 1 2; do
  for shape in "1 4" "1 8" "2 4" "2 2"; do
    set -- $shape
    echo -n "lpr=$1 batch=$2 " >> "$OUT/ab_spmv_shape.log"
    PNP_SPMV_LPR=$1 PNP_SPMV_BATCH=$2 timeout -k 10 120 python tools/ab_asm.py >> "$OUT/ab_spmv_shape.log" 2>&1 || exit $?
  done
done
PNP_SPMV_LPR=2 timeout -k 10 600 python -m pytest tests -q -m gpu -k "bicgstab or linear or newton or spmv or cg" > "$OUT/tests_lpr2.log" 2>&1
