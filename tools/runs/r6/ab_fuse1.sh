#!/bin/bash
# round 6: colour 1 of the second half step's forward sweep inside the BiCGSTAB update (PNP_FUSE1,
# default on) against its own colour launch: bit-for-bit hashes, the ILU variant tests, then
# tools/time_bicg.py at configs 3 and 5 interleaved three times, then the full GPU suite
# record: the colour-1 fusion (PNP_FUSE1) was reverted after this A/B
set -u
OUT=gpurun_out/$1; mkdir -p "$OUT"; : > "$OUT/ab_fuse1.log"
fatal() { case $1 in 124|134|137|139) return 0;; esac; [ "$1" -gt 128 ] && return 0; return 1; }
timeout -k 10 200 python tools/ilu_hash.py > "$OUT/hash_on.json" 2>&1 || exit 1
PNP_FUSE1=0 timeout -k 10 200 python tools/ilu_hash.py > "$OUT/hash_off.json" 2>&1 || exit 1
cmp "$OUT/hash_on.json" "$OUT/hash_off.json" && echo "bitwise: same" || echo "bitwise: DIFFERENT"
for i in 1 2 3; do
  for v in "PNP_FUSE1=1" "PNP_FUSE1=0"; do
    echo "== $v" >> "$OUT/ab_fuse1.log"
    env $v timeout -k 10 200 python tools/time_bicg.py 3,5 100 >> "$OUT/ab_fuse1.log" 2>&1; rc=$?; fatal $rc && exit 1
  done
done
timeout -k 10 700 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -rf > "$OUT/tests.log" 2>&1; rc=$?; echo "tests rc=$rc"; tail -2 "$OUT/tests.log"; fatal $rc && exit 1
exit 0
