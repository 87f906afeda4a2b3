#!/bin/bash
# round 6: the LDS sweeps' staged entries issued together per thread (ILU_SU, build flag: 4 the
# default in-tree, 2 and 8 in dune-pnp_amd/ab/lib_su{2,8}.so from tools/build_ab.sh),
# tools/time_bicg.py at configs 3 and 5, interleaved twice
set -u
OUT=gpurun_out/$1; mkdir -p "$OUT"; : > "$OUT/ab_su.log"
fatal() { case $1 in 124|134|137|139) return 0;; esac; [ "$1" -gt 128 ] && return 0; return 1; }
for i in 1 2; do
  for v in "PNP_AB=su4" "PNP_AMD_LIB=dune-pnp_amd/ab/lib_su2.so" "PNP_AMD_LIB=dune-pnp_amd/ab/lib_su8.so"; do
    echo "== $v" >> "$OUT/ab_su.log"
    env $v timeout -k 10 200 python tools/time_bicg.py 3,5 100 >> "$OUT/ab_su.log" 2>&1; rc=$?; fatal $rc && exit 1
  done
done
exit 0
