#!/bin/bash
# A/B: spatial XCD block map for assembly / SpMV (PNP_BLKMAP=1 default) vs plain order
set -u
OUT=gpurun_out/$1; mkdir -p "$OUT"; : > "$OUT/ab_blkmap.log"
for i in 1 2 3; do
  for v in 1 0; do
    echo -n "blkmap=$v " >> "$OUT/ab_blkmap.log"
    PNP_BLKMAP=$v timeout -k 10 120 python tools/ab_asm.py >> "$OUT/ab_blkmap.log" 2>&1 || exit $?
  done
done
