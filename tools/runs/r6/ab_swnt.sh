#!/bin/bash
# round 6: the sweeps' factor loads non-temporal (PNP_SWEEP_NT=1, the default) or plain (0) with
# the 14-B bf16 records (a runtime knob), tools/time_bicg.py at configs 3 and 5, interleaved twice
set -u
OUT=gpurun_out/$1; mkdir -p "$OUT"; : > "$OUT/ab_swnt.log"
fatal() { case $1 in 124|134|137|139) return 0;; esac; [ "$1" -gt 128 ] && return 0; return 1; }
for i in 1 2; do
  for v in "PNP_SWEEP_NT=1" "PNP_SWEEP_NT=0"; do
    echo "== $v" >> "$OUT/ab_swnt.log"
    env $v timeout -k 10 200 python tools/time_bicg.py 3,5 100 >> "$OUT/ab_swnt.log" 2>&1; rc=$?; fatal $rc && exit 1
  done
done
exit 0
