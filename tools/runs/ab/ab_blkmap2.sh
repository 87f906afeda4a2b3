#!/bin/bash
# A/B: spatial block map on/off (PNP_BLKMAP) with the current kernels
set -u
OUT=gpurun_out/$1; mkdir -p "$OUT"; : > "$OUT/ab_blkmap2.log"
for i in 1 2 3; do
  for bm in 1 0; do
    echo -n "blkmap=$bm " >> "$OUT/ab_blkmap2.log"
    PNP_BLKMAP=$bm timeout -k 10 120 python tools/ab_asm.py >> "$OUT/ab_blkmap2.log" 2>&1 || exit $?
  done
done
