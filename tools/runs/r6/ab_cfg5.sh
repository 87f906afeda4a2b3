#!/bin/bash
# round 6: config-5 SpMV / ILU(0) shape knobs (tools/time_bicg.py 5), interleaved twice
set -u
OUT=gpurun_out/$1; mkdir -p "$OUT"; : > "$OUT/ab_cfg5.log"
fatal() { case $1 in 124|134|137|139) return 0;; esac; [ "$1" -gt 128 ] && return 0; return 1; }
for i in 1 2; do
  for v in "PNP_AB=base" "PNP_SPMV_LDS=0" "PNP_SPMV_LDS=0 PNP_SPMV_BATCH=4" "PNP_ILU_LDS_B=2" "PNP_ILU_LDS_B=4"; do
    echo "== $v" >> "$OUT/ab_cfg5.log"
    env $v timeout -k 10 150 python tools/time_bicg.py 5 100 >> "$OUT/ab_cfg5.log" 2>&1; rc=$?; fatal $rc && exit 1
  done
done
exit 0
