#!/bin/bash
# Interleaved A/B over library builds and environment settings on tools/ab_asm.py (one process
# per entry, 2 rounds).  usage: tools/ab_libs_env.sh <tag> "<lib|-> <VAR=v ...>" ...
#   lib "-" = the in-tree libpnp_amd.so, else dune-pnp_amd/ab/lib_<lib>.so
set -u
OUT=gpurun_out/$1; shift
mkdir -p "$OUT"; : > "$OUT/ab.log"
for round in 1 2; do
  for entry in "$@"; do
    lib=${entry%% *}
    envs=${entry#"$lib"}
    if [ "$lib" = "-" ]; then libenv=""; else libenv="PNP_AMD_LIB=dune-pnp_amd/ab/lib_$lib.so"; fi
    echo -n "lib=$lib $envs: " >> "$OUT/ab.log"
    env $libenv $envs timeout -k 10 120 python tools/ab_asm.py >> "$OUT/ab.log" 2>&1 || exit $?
  done
done
