#!/bin/bash
# A/B: assembly with register-resident fan columns (default) vs the index-load path
set -u
OUT=gpurun_out/$1; mkdir -p "$OUT"; : > "$OUT/ab_fanr.log"
for i in 1 2 3; do
  for v in ${MODES:-1 0}; do
    PNP_ASM_FANR=$v timeout -k 10 120 python tools/ab_asm.py >> "$OUT/ab_fanr.log" 2>&1 || exit $?
  done
done
