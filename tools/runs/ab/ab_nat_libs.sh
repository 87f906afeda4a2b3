#!/bin/bash
# A/B of library builds on the natural-order SSOR: tools/bench_ssor_natural.py (pore_pnp k=4, PB and
# PNP) once per build, interleaved twice.  usage: tools/ab_nat_libs.sh <tag> <lib>...  (lib "-" =
# in-tree, else dune-pnp_amd/ab/lib_<lib>.so)
set -u
OUT=gpurun_out/$1; shift; mkdir -p "$OUT"; : > "$OUT/ab.log"
for i in 1 2; do
  for lib in "$@"; do
    if [ "$lib" = "-" ]; then libenv=""; else libenv="PNP_AMD_LIB=dune-pnp_amd/ab/lib_$lib.so"; fi
    echo "== $lib round $i" >> "$OUT/ab.log"
    env $libenv timeout -k 10 200 python tools/bench_ssor_natural.py 4 >> "$OUT/ab.log" 2>&1 || exit $?
  done
done
