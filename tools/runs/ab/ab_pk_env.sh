#!/bin/bash
# A/B of an environment knob on the P_k assembly: the bitwise P_k tests, then tools/bench_pk.py
# (pore_pnp k=3, degrees 2 and 3) with VAR=1 and VAR=0 interleaved twice.
# usage: tools/ab_pk_env.sh <tag> <VAR>
set -u
OUT=gpurun_out/$1; VAR=$2; mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest -q --timeout 250 --timeout-method thread tests/test_gpu_pk_res2.py > "$OUT/pk_tests.log" 2>&1 || exit $?
for i in 1 2; do
  for v in 1 0; do
    env $VAR=$v PNP_PK_NO_SOLVE=1 timeout -k 10 200 python tools/bench_pk.py 3 2 3 > "$OUT/pk_${VAR}_${v}_$i.log" 2>&1 || exit $?
  done
done
