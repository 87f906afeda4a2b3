#!/bin/bash
# round 6: write-through (sc1) vector stores in the BiCGSTAB kernels (VEC_WT, in-tree default)
# against plain stores (dune-pnp_amd/ab/lib_nowt.so): bit-for-bit hashes, tools/time_bicg.py at
# configs 3 and 5 interleaved three times, the in-situ assembly probe, then the full GPU suite
# record: the write-through stores (VEC_WT; A/B lib: tools/build_ab.sh nowt -DVEC_WT=0) were
# reverted after this A/B
set -u
OUT=gpurun_out/$1; mkdir -p "$OUT"; : > "$OUT/ab_wt.log"
fatal() { case $1 in 124|134|137|139) return 0;; esac; [ "$1" -gt 128 ] && return 0; return 1; }
timeout -k 10 200 python tools/ilu_hash.py > "$OUT/hash_wt.json" 2>&1 || exit 1
PNP_AMD_LIB=dune-pnp_amd/ab/lib_nowt.so timeout -k 10 200 python tools/ilu_hash.py > "$OUT/hash_plain.json" 2>&1 || exit 1
cmp "$OUT/hash_wt.json" "$OUT/hash_plain.json" && echo "bitwise: same" || echo "bitwise: DIFFERENT"
for i in 1 2 3; do
  for v in "PNP_AB=wt" "PNP_AMD_LIB=dune-pnp_amd/ab/lib_nowt.so"; do
    echo "== $v" >> "$OUT/ab_wt.log"
    env $v timeout -k 10 200 python tools/time_bicg.py 3,5 100 >> "$OUT/ab_wt.log" 2>&1; rc=$?; fatal $rc && exit 1
  done
done
for v in "PNP_AB=wt" "PNP_AMD_LIB=dune-pnp_amd/ab/lib_nowt.so"; do
  echo "== insitu $v" >> "$OUT/ab_wt.log"
  env $v timeout -k 10 200 python tools/insitu_probe.py >> "$OUT/ab_wt.log" 2>&1; rc=$?; fatal $rc && exit 1
done
timeout -k 10 700 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -rf > "$OUT/tests.log" 2>&1; rc=$?; echo "tests rc=$rc"; tail -2 "$OUT/tests.log"; fatal $rc && exit 1
exit 0
