#!/bin/bash
# round 6: the three-plane bf16 PNP block (ILU_BF16_B7=2, dune-pnp_amd/ab/lib_p3.so, built with
# tools/build_ab.sh-style flags) against the two-plane one (in-tree): bit-for-bit hashes, then
# tools/time_bicg.py at configs 3 and 5 interleaved three times
# record: the three-plane form (ILU_BF16_B7=2) was reverted after this A/B
set -u
OUT=gpurun_out/$1; mkdir -p "$OUT"; : > "$OUT/ab_p3.log"
fatal() { case $1 in 124|134|137|139) return 0;; esac; [ "$1" -gt 128 ] && return 0; return 1; }
timeout -k 10 200 python tools/ilu_hash.py > "$OUT/hash_b7.json" 2>&1 || exit 1
PNP_AMD_LIB=dune-pnp_amd/ab/lib_p3.so timeout -k 10 200 python tools/ilu_hash.py > "$OUT/hash_p3.json" 2>&1 || exit 1
cmp "$OUT/hash_b7.json" "$OUT/hash_p3.json" && echo "bitwise: same" || echo "bitwise: DIFFERENT"
for i in 1 2 3; do
  for v in "PNP_AMD_LIB=dune-pnp_amd/ab/lib_p3.so" "PNP_AB=b7"; do
    echo "== $v" >> "$OUT/ab_p3.log"
    env $v timeout -k 10 200 python tools/time_bicg.py 3,5 100 >> "$OUT/ab_p3.log" 2>&1; rc=$?; fatal $rc && exit 1
  done
done
exit 0
