#!/bin/bash
# Interleaved A/B of env-knob variants in separate processes of one GPU session.
# usage: tools/ab_knobs.sh <tag> "<env assignments A>" "<env assignments B>" ...
set -u
OUT=gpurun_out/$1; shift; mkdir -p "$OUT"; : > "$OUT/ab.log"
for i in 1 2 3; do
  for v in "$@"; do
    env $v timeout -k 10 150 python tools/ab_asm.py >> "$OUT/ab.log" 2>&1 || { echo "fail rc=$? ($v)" >> "$OUT/ab.log"; exit 1; }
  done
done
cat "$OUT/ab.log"
