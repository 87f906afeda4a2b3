#!/bin/bash
# round 6: the 14-B bfloat16 PNP block record (ILU_BF16_B7, in-tree default) against the 16-B one
# (dune-pnp_amd/ab/lib_b16.so): the full GPU suite, bit-for-bit hashes of both, then
# tools/time_bicg.py at configs 3 and 5, interleaved three times
# the A/B lib first: tools/build_ab.sh b16 "-DILU_BF16_B7=0" (the 14-B layout is the default)
set -u
OUT=gpurun_out/$1; mkdir -p "$OUT"; : > "$OUT/ab_b7.log"
fatal() { case $1 in 124|134|137|139) return 0;; esac; [ "$1" -gt 128 ] && return 0; return 1; }
timeout -k 10 700 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -rf > "$OUT/tests.log" 2>&1; rc=$?; echo "tests rc=$rc"; tail -2 "$OUT/tests.log"; fatal $rc && exit 1
timeout -k 10 200 python tools/ilu_hash.py > "$OUT/hash_b7.json" 2>&1 || exit 1
PNP_AMD_LIB=dune-pnp_amd/ab/lib_b16.so timeout -k 10 200 python tools/ilu_hash.py > "$OUT/hash_b16.json" 2>&1 || exit 1
cmp "$OUT/hash_b7.json" "$OUT/hash_b16.json" && echo "bitwise: same" || echo "bitwise: DIFFERENT"
for i in 1 2 3; do
  for v in "PNP_AB=b7" "PNP_AMD_LIB=dune-pnp_amd/ab/lib_b16.so"; do
    echo "== $v" >> "$OUT/ab_b7.log"
    env $v timeout -k 10 200 python tools/time_bicg.py 3,5 100 >> "$OUT/ab_b7.log" 2>&1; rc=$?; fatal $rc && exit 1
  done
done
exit 0
