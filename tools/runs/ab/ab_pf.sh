#!/bin/bash
# A/B: assembly gather prefetch distance (PNP_ASM_PF 1 / 2), plus the assembly GPU tests at PF=2
set -u
OUT=gpurun_out/$1; mkdir -p "$OUT"; : > "$OUT/ab_pf.log"
for i in 1 2 3; do
  for pf in 1 2; do
    echo -n "pf=$pf " >> "$OUT/ab_pf.log"
    PNP_ASM_PF=$pf timeout -k 10 120 python tools/ab_asm.py >> "$OUT/ab_pf.log" 2>&1 || exit $?
  done
done
PNP_ASM_PF=2 timeout -k 10 600 python -m pytest tests -q -m gpu -k "assembl or residual or jacobian or newton" > "$OUT/tests_pf2.log" 2>&1
