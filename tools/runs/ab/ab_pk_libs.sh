#!/bin/bash
# A/B of library builds on the P_k assembly: tools/bench_pk.py (pore_pnp k=3, degrees 2 and 3)
# once per build, interleaved twice.  usage: tools/ab_pk_libs.sh <tag> <lib>...  (lib "-" = in-tree,
# else dune-pnp_amd/ab/lib_<lib>.so)
set -u
OUT=gpurun_out/$1; shift; mkdir -p "$OUT"
for i in 1 2; do
  for lib in "$@"; do
    if [ "$lib" = "-" ]; then libenv=""; else libenv="PNP_AMD_LIB=dune-pnp_amd/ab/lib_$lib.so"; fi
    env $libenv PNP_PK_NO_SOLVE=1 timeout -k 10 200 python tools/bench_pk.py 3 2 3 > "$OUT/pk_${lib}_$i.log" 2>&1 || exit $?
  done
done
