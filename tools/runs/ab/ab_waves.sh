#!/bin/bash
# A/B: assembly occupancy variant (PNP_ASM_WAVES=3 default vs 4)
set -u
OUT=gpurun_out/$1; mkdir -p "$OUT"; : > "$OUT/ab_waves.log"
for i in 1 2 3; do
  for w in 3 4; do
    PNP_ASM_WAVES=$w timeout -k 10 120 python tools/ab_asm.py >> "$OUT/ab_waves.log" 2>&1 || exit $?
  done
done
