#!/bin/bash
# A/B of library builds on the AMG-preconditioned PNP Newton (tools/time_amg_graph.py, config 3),
# once per build, interleaved twice.  usage: tools/ab_amg_libs.sh <tag> <lib>...  (lib "-" =
# in-tree, else dune-pnp_amd/ab/lib_<lib>.so)
set -u
OUT=gpurun_out/$1; shift; mkdir -p "$OUT"; : > "$OUT/ab.log"
for i in 1 2; do
  for lib in "$@"; do
    if [ "$lib" = "-" ]; then libenv=""; else libenv="PNP_AMD_LIB=dune-pnp_amd/ab/lib_$lib.so"; fi
    echo "== $lib round $i" >> "$OUT/ab.log"
    env $libenv timeout -k 10 200 python tools/time_amg_graph.py >> "$OUT/ab.log" 2>&1 || exit $?
  done
done
