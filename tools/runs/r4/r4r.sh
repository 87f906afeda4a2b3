#!/bin/bash
# chain kernel, lead 2 (the default now): bitwise tests; A/B against history 8 and lead 4 at three
# thresholds, interleaved twice
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r4r; mkdir -p $O
export TMPDIR=/tmp
PNP_NAT_CHAIN=8192 timeout -k 10 300 python -u -m pytest tests/test_gpu_ssor_natural.py -x -q --timeout 200 --timeout-method thread > $O/nat_tests_chain.log 2>&1; rc=$?; echo "nat tests rc=$rc"
[ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python -u -m pytest tests/test_gpu_ssor_chain.py -x -q --timeout 800 --timeout-method thread > $O/chain_tests.log 2>&1; rc=$?; echo "chain tests rc=$rc"
[ $rc -ne 0 ] && exit $rc
for i in 1 2; do
  for lib in - ch8 cd4; do
    if [ "$lib" = "-" ]; then libenv=""; else libenv="PNP_AMD_LIB=dune-pnp_amd/ab/lib_$lib.so"; fi
    for T in 4096 8192 16384; do
      echo "== $lib chain $T round $i" >> $O/ab.log
      env $libenv PNP_NAT_CHAIN=$T timeout -k 10 200 python tools/bench_ssor_natural.py 4 >> $O/ab.log 2>&1 || exit $?
    done
  done
done
