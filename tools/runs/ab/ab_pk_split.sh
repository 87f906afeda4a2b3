#!/bin/bash
# the P_k Jacobian gather split (PNP_PK_SPLIT) on / off: tools/bench_pk.py (pore_pnp k=3, degrees 2
# and 3) interleaved twice, after the bitwise test of the two-pass assembly.  usage: tools/ab_pk_split.sh <tag>
set -u
OUT=gpurun_out/$1; mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest -q --timeout 250 --timeout-method thread tests/test_gpu_pk_res2.py > "$OUT/pk_tests.log" 2>&1 || exit $?
for i in 1 2; do
  for v in 1 0; do
    PNP_PK_SPLIT=$v PNP_PK_NO_SOLVE=1 timeout -k 10 200 python tools/bench_pk.py 3 2 3 > "$OUT/pk_split_${v}_$i.log" 2>&1 || exit $?
  done
done
