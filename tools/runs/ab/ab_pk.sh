#!/bin/bash
# P_k assembly A/B: the in-tree library vs dune-pnp_amd/ab/lib_pkbase.so (tools/bench_pk.py,
# pore_pnp k=3, degrees 2 and 3), after the P_k GPU tests.  usage: tools/ab_pk.sh <tag>
set -u
OUT=gpurun_out/$1; mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_gpu_pk.py > "$OUT/pk_tests.log" 2>&1 || exit $?
for i in 1 2; do
  PNP_PK_NO_SOLVE=1 timeout -k 10 200 python tools/bench_pk.py 3 2 3 > "$OUT/pk_new_$i.log" 2>&1 || exit $?
  PNP_PK_NO_SOLVE=1 PNP_AMD_LIB=dune-pnp_amd/ab/lib_pkbase.so timeout -k 10 200 python tools/bench_pk.py 3 2 3 > "$OUT/pk_base_$i.log" 2>&1 || exit $?
done
