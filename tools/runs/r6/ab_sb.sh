#!/bin/bash
# round 6: the partition edge-case tests, then the LDS SpMV's four-slot step (PNP_SPMV_LDS_SB=4)
# against the pairs: bitwise test, then tools/time_bicg.py at configs 3 and 5, interleaved 3 times
# record: the four-slot SpMV step (PNP_SPMV_LDS_SB) was reverted after this A/B
set -u
OUT=gpurun_out/$1; mkdir -p "$OUT"; : > "$OUT/ab_sb.log"
fatal() { case $1 in 124|134|137|139) return 0;; esac; [ "$1" -gt 128 ] && return 0; return 1; }
timeout -k 10 400 python -u -m pytest -x -v --timeout 380 --timeout-method thread \
  tests/test_gpu_multirank.py -k "vertex or vertices or spmv" tests/test_gpu_spmv_lds.py > "$OUT/tests.log" 2>&1 || exit 1
for i in 1 2 3; do
  for v in "PNP_SPMV_LDS_SB=2" "PNP_SPMV_LDS_SB=4"; do
    echo "== $v" >> "$OUT/ab_sb.log"
    env $v timeout -k 10 200 python tools/time_bicg.py 3,5 100 >> "$OUT/ab_sb.log" 2>&1; rc=$?; fatal $rc && exit 1
  done
done
exit 0
