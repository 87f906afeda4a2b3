#!/bin/bash
# round 6: does the solve's non-temporal matrix / factor loading decide where the in-situ
# assembly's write stream lands?  In-situ assembly (tools/ab_newton_asm.py) and BiCGSTAB
# (tools/time_bicg.py 3) under the NT knobs, interleaved twice
set -u
OUT=gpurun_out/$1; mkdir -p "$OUT"; : > "$OUT/ab_nt.log"
fatal() { case $1 in 124|134|137|139) return 0;; esac; [ "$1" -gt 128 ] && return 0; return 1; }
for i in 1 2; do
  for v in "PNP_AB=base" "PNP_SPMV_NT=0" "PNP_SWEEP_NT=0" "PNP_SPMV_NT=0 PNP_SWEEP_NT=0"; do
    echo "== $v" >> "$OUT/ab_nt.log"
    env $v timeout -k 10 120 python tools/ab_newton_asm.py >> "$OUT/ab_nt.log" 2>&1; rc=$?; fatal $rc && exit 1
    env $v timeout -k 10 120 python tools/time_bicg.py 3 200 >> "$OUT/ab_nt.log" 2>&1; rc=$?; fatal $rc && exit 1
  done
done
exit 0
