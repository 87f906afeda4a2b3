#!/bin/bash
# A/B of two builds of libpnp_amd.so (dune-pnp_amd/ab/lib_base.so vs lib_new.so), interleaved
set -u
OUT=gpurun_out/$1; mkdir -p "$OUT"; : > "$OUT/ab_lib.log"
for i in 1 2 3; do
  for v in new base; do
    echo -n "$v " >> "$OUT/ab_lib.log"
    PNP_AMD_LIB=dune-pnp_amd/ab/lib_$v.so timeout -k 10 120 python tools/ab_asm.py >> "$OUT/ab_lib.log" 2>&1 || exit $?
  done
done
