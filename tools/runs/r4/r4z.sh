#!/bin/bash
# natural SSOR: 4 lanes per row (16-row units) and 6/8 head workgroups per CU, A/B interleaved
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r4z; mkdir -p $O
export TMPDIR=/tmp
PNP_AMD_LIB=dune-pnp_amd/ab/lib_kl4.so timeout -k 10 300 python -u -m pytest tests/test_gpu_ssor_natural.py -x -q --timeout 200 --timeout-method thread > $O/nat_tests_kl4.log 2>&1; rc=$?; echo "nat tests kl4 rc=$rc"
[ $rc -ne 0 ] && exit $rc
for i in 1 2; do
  for lib in - kl4; do
    if [ "$lib" = "-" ]; then libenv=""; else libenv="PNP_AMD_LIB=dune-pnp_amd/ab/lib_$lib.so"; fi
    for W in 4 8; do
      for C in default 0; do
        if [ "$C" = "default" ]; then cenv=""; else cenv="PNP_NAT_CHAIN=$C"; fi
        echo "== $lib wg $W chain $C round $i" >> $O/ab.log
        env $libenv $cenv PNP_NAT_FLOW_WG_PER_CU=$W timeout -k 10 200 python tools/bench_ssor_natural.py 4 >> $O/ab.log 2>&1 || exit $?
      done
    done
  done
done
