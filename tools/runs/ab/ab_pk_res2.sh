#!/bin/bash
# two-pass P_k residual and Jacobian vs the row walk (PNP_PK_RES2, PNP_PK_JAC2): the P_k GPU tests, then tools/bench_pk.py
# (pore_pnp k=3, degrees 2 and 3) with the knob on / off, twice each.  usage: tools/ab_pk_res2.sh <tag>
set -u
OUT=gpurun_out/$1; mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_pk_res2.py tests/test_gpu_pk.py > "$OUT/pk_tests.log" 2>&1 || exit $?
for i in 1 2; do
  for v in 1 0; do
    PNP_PK_RES2=$v PNP_PK_JAC2=$v PNP_PK_NO_SOLVE=1 timeout -k 10 200 python tools/bench_pk.py 3 2 3 > "$OUT/pk_res2_${v}_$i.log" 2>&1 || exit $?
  done
done
