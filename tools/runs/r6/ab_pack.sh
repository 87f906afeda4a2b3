#!/bin/bash
# round 6: packed ILU(0) row metadata (PNP_ILU_PACK, default on) against the byte arrays, the
# ILU LDS variant tests first, then tools/time_bicg.py at configs 3 and 5, interleaved three times
# record: the packed-metadata variant (PNP_ILU_PACK) was reverted after this A/B
set -u
OUT=gpurun_out/$1; mkdir -p "$OUT"; : > "$OUT/ab_pack.log"
fatal() { case $1 in 124|134|137|139) return 0;; esac; [ "$1" -gt 128 ] && return 0; return 1; }
timeout -k 10 400 python -u -m pytest -x -v --timeout 380 --timeout-method thread \
  tests/test_gpu_ilu_lds.py > "$OUT/tests.log" 2>&1 || exit 1
for i in 1 2 3; do
  for v in "PNP_ILU_PACK=1" "PNP_ILU_PACK=0"; do
    echo "== $v" >> "$OUT/ab_pack.log"
    env $v timeout -k 10 200 python tools/time_bicg.py 3,5 100 >> "$OUT/ab_pack.log" 2>&1; rc=$?; fatal $rc && exit 1
  done
done
exit 0
