#!/bin/bash
# Interleaved A/B of env-knob variants on the config-5 assembly (tools/prof_cfg5.py k=6).
# usage: tools/ab_cfg5.sh <tag> "<env A>" "<env B>" ...
set -u
OUT=gpurun_out/$1; shift; mkdir -p "$OUT"; : > "$OUT/ab.log"
for i in 1 2; do
  for v in "$@"; do
    echo -n "$v: " >> "$OUT/ab.log"
    env $v timeout -k 10 150 python tools/prof_cfg5.py 6 20 >> "$OUT/ab.log" 2>&1 || { echo "fail rc=$? ($v)" >> "$OUT/ab.log"; exit 1; }
  done
done
cat "$OUT/ab.log"
