#!/bin/bash
# round 6: the LDS sweeps' slot batch with the 14-B bf16 records (PNP_ILU_LDS_B = 2 default, 3,
# 4), tools/time_bicg.py at configs 3 and 5, interleaved twice
set -u
OUT=gpurun_out/$1; mkdir -p "$OUT"; : > "$OUT/ab_batch.log"
fatal() { case $1 in 124|134|137|139) return 0;; esac; [ "$1" -gt 128 ] && return 0; return 1; }
for i in 1 2; do
  for v in "PNP_ILU_LDS_B=2" "PNP_ILU_LDS_B=3" "PNP_ILU_LDS_B=4"; do
    echo "== $v" >> "$OUT/ab_batch.log"
    env $v timeout -k 10 200 python tools/time_bicg.py 3,5 100 >> "$OUT/ab_batch.log" 2>&1; rc=$?; fatal $rc && exit 1
  done
done
exit 0
