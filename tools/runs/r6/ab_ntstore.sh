#!/bin/bash
# round 6: non-temporal vector stores in the BiCGSTAB kernels (VEC_NT, in-tree)
# against plain stores (dune-pnp_amd/ab/lib_plain.so): bit-for-bit hashes, tools/time_bicg.py at
# configs 3 and 5 interleaved three times, the in-situ assembly probe, then the full GPU suite
# record: the non-temporal stores (VEC_NT; A/B lib: tools/build_ab.sh plain -DVEC_NT=0) were
# reverted after this A/B
set -u
OUT=gpurun_out/$1; mkdir -p "$OUT"; : > "$OUT/ab_nt.log"
fatal() { case $1 in 124|134|137|139) return 0;; esac; [ "$1" -gt 128 ] && return 0; return 1; }
timeout -k 10 200 python tools/ilu_hash.py > "$OUT/hash_nt.json" 2>&1 || exit 1
PNP_AMD_LIB=dune-pnp_amd/ab/lib_plain.so timeout -k 10 200 python tools/ilu_hash.py > "$OUT/hash_plain.json" 2>&1 || exit 1
cmp "$OUT/hash_nt.json" "$OUT/hash_plain.json" && echo "bitwise: same" || echo "bitwise: DIFFERENT"
for i in 1 2 3; do
  for v in "PNP_AB=nt" "PNP_AMD_LIB=dune-pnp_amd/ab/lib_plain.so"; do
    echo "== $v" >> "$OUT/ab_nt.log"
    env $v timeout -k 10 200 python tools/time_bicg.py 3,5 100 >> "$OUT/ab_nt.log" 2>&1; rc=$?; fatal $rc && exit 1
  done
done
for v in "PNP_AB=nt" "PNP_AMD_LIB=dune-pnp_amd/ab/lib_plain.so"; do
  echo "== insitu $v" >> "$OUT/ab_nt.log"
  env $v timeout -k 10 200 python tools/insitu_probe.py >> "$OUT/ab_nt.log" 2>&1; rc=$?; fatal $rc && exit 1
done
timeout -k 10 700 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -rf > "$OUT/tests.log" 2>&1; rc=$?; echo "tests rc=$rc"; tail -2 "$OUT/tests.log"; fatal $rc && exit 1
exit 0
