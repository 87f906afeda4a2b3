#!/bin/bash
# A/B: non-temporal L/U value loads in the sweeps (PNP_SWEEP_NT)
set -u
OUT=gpurun_out/$1; mkdir -p "$OUT"; : > "$OUT/ab_sweep_nt.log"
for i in 1 2 3; do
  for nt in 0 1; do
    echo -n "sweep_nt=$nt " >> "$OUT/ab_sweep_nt.log"
    PNP_SWEEP_NT=$nt timeout -k 10 120 python tools/ab_asm.py >> "$OUT/ab_sweep_nt.log" 2>&1 || exit $?
  done
done
